"""Client of the Brain service + a master-side resource optimizer backed by
it (falls back to the local heuristics when the Brain is unreachable).

Parity: reference ``dlrover/python/brain/client.py`` (``BrainClient``:
``report_metrics`` / ``get_job_metrics`` / ``request_optimization`` /
``report_training_hyper_params`` ...) and
``dlrover/python/master/resource/brain_optimizer.py``.
"""

import json
import time
from typing import Any, Dict, List, Optional

from ..common.constants import NodeType
from ..common.log import logger
from ..common.node import JobResource, NodeGroupResource, NodeResource
from ..common.rpc import RpcClient, addr_connected
from ..master.autoscale import JobResourceOptimizer, ResourcePlan
from .service import MetricsType


class BrainClient:
    def __init__(self, addr: str, job_uuid: str = "", job_name: str = "", user: str = "", timeout: float = 5.0):
        self.addr = addr
        self.job_uuid, self.job_name, self.user = job_uuid, job_name, user
        self._rpc = RpcClient(addr, timeout=timeout) if addr else None

    def available(self) -> bool:
        return self._rpc is not None and addr_connected(self.addr)

    def _metrics(self, metrics_type: str, metrics: Dict[str, Any]) -> Dict[str, Any]:
        return {"job_uuid": self.job_uuid, "job_name": self.job_name, "user": self.user,
                "metrics_type": metrics_type, "metrics": metrics, "ts": time.time()}

    def report_metrics(self, metrics_type: str, metrics: Dict[str, Any]) -> bool:
        res = json.loads(self._rpc.report(json.dumps(self._metrics(metrics_type, metrics)).encode()))
        return bool(res.get("success"))

    def report_resource_usage(self, node_type: str, node_name: str, cpu: float, cpu_used: float, memory_mb: int,
                              memory_used_mb: int) -> bool:
        return self.report_metrics(MetricsType.RESOURCE_USAGE, {
            "node_type": node_type, "node_name": node_name, "cpu": cpu, "cpu_used": cpu_used,
            "memory_mb": memory_mb, "memory_used_mb": memory_used_mb})

    def report_speed(self, worker_num: int, speed: float) -> bool:
        return self.report_metrics(MetricsType.SPEED, {"worker_num": worker_num, "speed": speed})

    def report_oom(self, node_type: str, memory_mb: int) -> bool:
        return self.report_metrics(MetricsType.OOM, {"node_type": node_type, "memory_mb": memory_mb})

    def report_training_hyper_params(self, batch_size: int, epoch: int = 0, max_steps: int = 0) -> bool:
        return self.report_metrics(MetricsType.HYPER_PARAMS,
                                   {"batch_size": batch_size, "epoch": epoch, "max_steps": max_steps})

    def get_job_metrics(self, job_uuid: Optional[str] = None, metrics_type: Optional[str] = None) -> List[Dict]:
        req = {"method": "get_job_metrics", "job_uuid": job_uuid or self.job_uuid, "metrics_type": metrics_type}
        res = json.loads(self._rpc.get(json.dumps(req).encode()))
        if not res.get("success"):
            raise RuntimeError(res.get("reason"))
        return res["result"]

    def request_optimization(self, opt_type: str, **config) -> Dict[str, Any]:
        req = dict(config, method="optimize", opt_type=opt_type, job_uuid=self.job_uuid, job_name=self.job_name)
        res = json.loads(self._rpc.get(json.dumps(req).encode()))
        if not res.get("success"):
            raise RuntimeError(res.get("reason"))
        return res["result"]

    def close(self):
        if self._rpc is not None:
            self._rpc.close()


class BrainResourceOptimizer(JobResourceOptimizer):
    """Worker resource plans from the Brain: initial resources on job
    creation, OOM memory bumps, running worker count from the speed curve."""

    def __init__(self, client: BrainClient, job_resource: JobResource, max_workers: int = 0, node_unit: int = 1):
        self.client = client
        self.job_resource = job_resource
        self.max_workers = max_workers
        self.node_unit = node_unit

    def _worker_group(self) -> NodeGroupResource:
        g = self.job_resource.get_node_group_resource(NodeType.WORKER)
        if g is None:
            g = NodeGroupResource(0, NodeResource())
            self.job_resource.node_group_resources[NodeType.WORKER] = g
        return g

    def init_job_resource(self) -> ResourcePlan:
        plan = ResourcePlan()
        try:
            r = self.client.request_optimization("job_create_resource").get("worker", {})
        except Exception as e:
            logger.warning(f"brain unavailable for the initial plan: {e}")
            return plan
        g = self._worker_group()
        res = NodeResource(cpu=r.get("cpu", g.node_resource.cpu), memory=r.get("memory_mb", g.node_resource.memory),
                           gpu_type=g.node_resource.gpu_type, gpu_num=g.node_resource.gpu_num)
        plan.node_group_resources[NodeType.WORKER] = NodeGroupResource(g.count, res)
        return plan

    def get_oom_resource_plan(self) -> ResourcePlan:
        plan = ResourcePlan()
        r = self.client.request_optimization("job_oom_resource").get(NodeType.WORKER, {})
        if r:
            g = self._worker_group()
            res = NodeResource(cpu=g.node_resource.cpu, memory=r["memory_mb"], gpu_type=g.node_resource.gpu_type,
                               gpu_num=g.node_resource.gpu_num)
            plan.node_group_resources[NodeType.WORKER] = NodeGroupResource(g.count, res)
        return plan

    def get_job_resource_plan(self) -> ResourcePlan:
        plan = ResourcePlan()
        g = self._worker_group()
        try:
            r = self.client.request_optimization("job_running_workers", max_workers=self.max_workers,
                                                 node_unit=self.node_unit, current_workers=g.count)
        except Exception as e:
            logger.warning(f"brain unavailable: {e}")
            return plan
        cnt = r.get("worker", {}).get("count")
        if cnt:
            plan.node_group_resources[NodeType.WORKER] = NodeGroupResource(int(cnt), g.node_resource)
        return plan
