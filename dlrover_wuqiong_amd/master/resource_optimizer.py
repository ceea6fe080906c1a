"""Job resource optimizer of the master ("single-job" optimize mode), and the
factory that picks it or the Brain service ("cluster" mode).

The local optimizer runs the SAME algorithms as the Brain service
(``brain/service.py:BrainOptimizer``) over an in-memory datastore that this
master's own monitors feed (resource usage, speed records, OOMs, job meta),
so a job without a Brain still gets history-free versions of every plan and
a job with one gets cross-job history -- one implementation, two scopes.

Stages (reference ``JobOptStage``):
  * ``job_create``      initial worker resources (AllReduce) or PS count /
                        resources (PS); GPU nodes also get their host memory
                        sized for flash-checkpoint shm slots;
  * ``ps_initial``      PS memory extrapolated from its early growth;
  * ``running``         AllReduce: worker count from the speed curve; PS: hot
                        PS CPU up, idle PS CPU down;
and OOM recovery plans (worker / PS memory x factor).  Every plan is clipped
to the job's ``ResourceLimits`` (per-node CPU / memory caps, worker count).

Parity: reference ``dlrover/python/master/resource/optimizer.py``
(``ResourcePlan``, ``ResourceOptimizer``, ``SimpleOptimizer``),
``resource/local_optimizer.py`` (``PSLocalOptimizer``: stages, speed ratio,
hot PS) and ``resource/brain_optimizer.py`` (``BrainResoureOptimizer``).
"""

import time
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from ..brain.service import BrainDatastore, BrainOptimizer, MetricsType
from ..common.constants import DistributionStrategy, NodeType
from ..common.log import logger
from ..common.node import NodeGroupResource, NodeResource
from .autoscale import ResourcePlan


class OptimizeStage:
    JOB_CREATE = "job_create"
    PS_INITIAL = "ps_initial"
    RUNNING = "running"


@dataclass
class ResourceLimits:
    cpu: float = 0.0          # per node, 0 = unlimited
    memory_mb: int = 0
    max_workers: int = 0
    max_ps: int = 0
    node_unit: int = 1        # worker counts rounded to this (whole TP/PP groups)


class ResourceOptimizer:
    def report(self, metrics_type: str, metrics: Dict[str, Any]):
        raise NotImplementedError

    def generate_opt_plan(self, stage: str, config: Optional[Dict] = None) -> ResourcePlan:
        raise NotImplementedError

    def generate_oom_recovery_plan(self, oom_node_type: str, memory_mb: int, stage: str = OptimizeStage.RUNNING
                                   ) -> ResourcePlan:
        raise NotImplementedError


class _AlgoOptimizer(ResourceOptimizer):
    """Plans from BrainOptimizer results (``_request`` supplies them)."""

    def __init__(self, job_uuid: str, job_name: str, limits: ResourceLimits, strategy: str):
        self.job_uuid, self.job_name = job_uuid, job_name
        self.limits = limits
        self.strategy = strategy

    def _request(self, opt_type: str, **cfg) -> Dict[str, Any]:
        raise NotImplementedError

    # --------------------------------------------------------------- clip
    def _res(self, cpu: float = 0.0, memory_mb: int = 0, gpu: int = 0) -> NodeResource:
        lim = self.limits
        if lim.cpu and cpu:
            cpu = min(cpu, lim.cpu)
        if lim.memory_mb and memory_mb:
            memory_mb = min(memory_mb, lim.memory_mb)
        return NodeResource(cpu=cpu, memory=int(memory_mb), gpu_num=gpu)

    def _count(self, n: int, node_type: str) -> int:
        cap = self.limits.max_workers if node_type == NodeType.WORKER else self.limits.max_ps
        if cap:
            n = min(n, cap)
        if node_type == NodeType.WORKER:
            u = max(1, self.limits.node_unit)
            n = max(u, n // u * u)
        return max(0, n)

    # -------------------------------------------------------------- plans
    def generate_opt_plan(self, stage: str, config: Optional[Dict] = None) -> ResourcePlan:
        cfg = dict(config or {})
        plan = ResourcePlan()
        ps = self.strategy == DistributionStrategy.PS
        try:
            if stage == OptimizeStage.JOB_CREATE:
                if ps:
                    r = self._request("job_ps_create_resource", **cfg).get("ps", {})
                    if r:
                        plan.node_group_resources[NodeType.PS] = NodeGroupResource(
                            self._count(int(r.get("count", 1)), NodeType.PS),
                            self._res(r.get("cpu", 0), r.get("memory_mb", 0)))
                w = self._request("job_create_resource", **cfg).get("worker", {})
                mem = int(w.get("memory_mb", 0))
                if cfg.get("ckpt_bytes_per_node"):
                    host = self._request("job_gpu_host_memory", **cfg).get("worker", {})
                    mem = max(mem, int(host.get("memory_mb", 0)))
                if w or mem:
                    plan.node_group_resources[NodeType.WORKER] = NodeGroupResource(
                        self._count(int(cfg.get("workers", 0)), NodeType.WORKER) if cfg.get("workers") else 0,
                        self._res(w.get("cpu", 0), mem, int(cfg.get("gpus_per_node", 0))))
            elif stage == OptimizeStage.PS_INITIAL:
                for name, r in self._request("job_ps_init_adjust_resource", **cfg).get("ps_nodes", {}).items():
                    plan.node_resources[name] = self._res(r.get("cpu", 0), r.get("memory_mb", 0))
            elif stage == OptimizeStage.RUNNING:
                if ps:
                    for opt in ("job_ps_resource_util", "job_hot_ps"):  # hot PS wins on a conflict
                        for name, r in self._request(opt, **cfg).get("ps_nodes", {}).items():
                            plan.node_resources[name] = self._res(r.get("cpu", 0), r.get("memory_mb", 0))
                else:
                    r = self._request("job_running_workers", max_workers=self.limits.max_workers,
                                      node_unit=self.limits.node_unit, **cfg)
                    cnt = r.get("worker", {}).get("count")
                    if cnt:
                        plan.node_group_resources[NodeType.WORKER] = NodeGroupResource(
                            self._count(int(cnt), NodeType.WORKER), NodeResource())
        except Exception as e:  # a failed optimisation is an empty plan, never a job failure
            logger.warning(f"resource optimizer: stage {stage} failed: {e}")
        return plan

    def generate_oom_recovery_plan(self, oom_node_type: str, memory_mb: int, stage: str = OptimizeStage.RUNNING
                                   ) -> ResourcePlan:
        self.report(MetricsType.OOM, {"node_type": oom_node_type, "memory_mb": int(memory_mb)})
        plan = ResourcePlan()
        try:
            if oom_node_type == NodeType.PS:
                r = self._request("job_ps_oom_resource").get("ps", {})
            elif stage == OptimizeStage.JOB_CREATE:
                r = self._request("job_worker_create_oom_resource").get("worker", {})
            else:
                r = self._request("job_oom_resource").get(oom_node_type, {})
        except Exception as e:
            logger.warning(f"resource optimizer: OOM plan failed: {e}")
            return plan
        if r.get("memory_mb"):
            plan.node_group_resources[oom_node_type] = NodeGroupResource(0, self._res(r.get("cpu", 0),
                                                                                     r["memory_mb"]))
        return plan


class LocalResourceOptimizer(_AlgoOptimizer):
    """Single-job mode: Brain algorithms over this master's own metrics."""

    def __init__(self, job_uuid: str, job_name: str, limits: Optional[ResourceLimits] = None,
                 strategy: str = DistributionStrategy.ALLREDUCE, **algo_kw):
        super().__init__(job_uuid, job_name, limits or ResourceLimits(), strategy)
        self.store = BrainDatastore(":memory:")
        self.algo = BrainOptimizer(self.store, **algo_kw)

    def report(self, metrics_type: str, metrics: Dict[str, Any]):
        self.store.persist({"job_uuid": self.job_uuid, "job_name": self.job_name, "metrics_type": metrics_type,
                            "metrics": dict(metrics), "ts": time.time()})

    def report_speed(self, worker_num: int, speed: float):
        self.report(MetricsType.SPEED, {"worker_num": int(worker_num), "speed": float(speed)})

    def _request(self, opt_type: str, **cfg) -> Dict[str, Any]:
        return self.algo.optimize(dict(cfg, opt_type=opt_type, job_uuid=self.job_uuid, job_name=self.job_name))


class BrainServiceOptimizer(_AlgoOptimizer):
    """Cluster mode: the Brain service's cross-job history; every metric is
    also kept locally so a Brain outage degrades to the local plans."""

    def __init__(self, client, limits: Optional[ResourceLimits] = None,
                 strategy: str = DistributionStrategy.ALLREDUCE):
        super().__init__(client.job_uuid, client.job_name, limits or ResourceLimits(), strategy)
        self.client = client
        self.local = LocalResourceOptimizer(client.job_uuid, client.job_name, self.limits, strategy)

    def report(self, metrics_type: str, metrics: Dict[str, Any]):
        self.local.report(metrics_type, metrics)
        try:
            self.client.report_metrics(metrics_type, metrics)
        except Exception as e:
            logger.warning(f"brain report failed: {e}")

    def _request(self, opt_type: str, **cfg) -> Dict[str, Any]:
        try:
            return self.client.request_optimization(opt_type, **cfg)
        except Exception as e:
            logger.warning(f"brain optimize {opt_type} failed ({e}); using the local optimizer")
            return self.local._request(opt_type, **cfg)


def new_resource_optimizer(optimize_mode: str, job_uuid: str, job_name: str,
                           limits: Optional[ResourceLimits] = None, strategy: str = DistributionStrategy.ALLREDUCE,
                           brain_addr: Optional[str] = None) -> ResourceOptimizer:
    if optimize_mode == "cluster" and brain_addr:
        from ..brain.client import BrainClient

        return BrainServiceOptimizer(BrainClient(brain_addr, job_uuid, job_name), limits, strategy)
    return LocalResourceOptimizer(job_uuid, job_name, limits, strategy)
