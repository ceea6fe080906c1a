"""Resource plans, job resource optimizers and job auto-scalers.

Parity: reference ``master/resource/job.py`` (``JobResourceOptimizer``,
``AllreduceJobResourceOptimizer``, ``PSJobResourceOptimizer``),
``resource/local_optimizer.py`` (heuristics when no Brain service) and
``master/node/job_auto_scaler.py`` (``JobAutoScaler`` :73,
``PSTrainingAutoScaler`` :98, ``AllreduceTrainingAutoScaler`` :254).

AllReduce (the GPU case): the optimizer plans the worker count from the
alive nodes plus the configured maximum, rounded down to ``node_unit``
(e.g. keep TP/PP groups whole); the auto-scaler periodically asks it for a
plan and scales up when nodes can be added (e.g. replaced nodes came back).
"""

import threading
import time
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from typing import Dict, Optional

from ..common.constants import NodeStatus, NodeType
from ..common.log import logger
from ..common.node import JobResource, NodeGroupResource, NodeResource
from .scaler import ScalePlan


@dataclass
class ResourcePlan:
    node_group_resources: Dict[str, NodeGroupResource] = field(default_factory=dict)
    node_resources: Dict[str, NodeResource] = field(default_factory=dict)

    def empty(self) -> bool:
        return not self.node_group_resources and not self.node_resources


class JobResourceOptimizer(ABC):
    @abstractmethod
    def get_job_resource_plan(self) -> ResourcePlan:
        ...


class AllreduceJobResourceOptimizer(JobResourceOptimizer):
    """Worker count = alive nodes (replaced nodes come back), raised to what
    the resource optimizer's speed curve recommends (``resource_optimizer``:
    ``master/resource_optimizer.py``; scale-up only while the marginal
    per-node throughput holds), capped at ``max_workers`` and whole
    ``node_unit`` groups."""

    def __init__(self, job_resource: JobResource, max_workers: int = 0, node_unit: int = 1,
                 resource_optimizer=None):
        self._job_resource = job_resource
        self._max_workers = max_workers or job_resource.worker_num
        self._node_unit = max(1, node_unit)
        self._alive_node_num = 0
        self.resource_optimizer = resource_optimizer

    def set_alive_node_num(self, n: int):
        self._alive_node_num = n

    def get_job_resource_plan(self) -> ResourcePlan:
        g = self._job_resource.get_node_group_resource(NodeType.WORKER) or NodeGroupResource()
        target = max(self._alive_node_num, g.count)
        if self.resource_optimizer is not None:
            from .resource_optimizer import OptimizeStage

            rp = self.resource_optimizer.generate_opt_plan(OptimizeStage.RUNNING,
                                                           {"current_workers": self._alive_node_num})
            rg = rp.node_group_resources.get(NodeType.WORKER)
            if rg is not None and rg.count > 0:
                target = max(self._alive_node_num, rg.count)
        target = min(self._max_workers, target)
        target = target // self._node_unit * self._node_unit
        plan = ResourcePlan()
        plan.node_group_resources[NodeType.WORKER] = NodeGroupResource(target, g.node_resource)
        return plan


class PSJobResourceOptimizer(JobResourceOptimizer):
    """Local heuristic (no Brain): give hot PS nodes more CPU, cut the CPU of
    nodes that stayed pending too long."""

    def __init__(self, job_resource: JobResource, cpu_util_threshold: float = 0.8, factor: float = 1.5):
        self._job_resource = job_resource
        self._threshold = cpu_util_threshold
        self._factor = factor

    def get_job_resource_plan(self, nodes=None) -> ResourcePlan:
        plan = ResourcePlan()
        for n in (nodes or []):
            if n.type != NodeType.PS or n.config_resource.cpu <= 0:
                continue
            if n.used_cpu / n.config_resource.cpu > self._threshold:
                r = NodeResource(cpu=n.config_resource.cpu * self._factor, memory=n.config_resource.memory)
                plan.node_resources[n.name] = r
        return plan


class JobAutoScaler(ABC):
    def __init__(self):
        self._suggested_stop = False

    def suggested_stop(self) -> bool:
        return self._suggested_stop

    @abstractmethod
    def start_auto_scaling(self):
        ...

    @abstractmethod
    def stop_auto_scaling(self):
        ...

    @abstractmethod
    def execute_job_optimization_plan(self, plan: ResourcePlan) -> ScalePlan:
        ...


class AllreduceTrainingAutoScaler(JobAutoScaler):
    def __init__(self, job_resource: JobResource, job_nodes, job_optimizer: AllreduceJobResourceOptimizer,
                 speed_monitor, worker_manager, node_scaler, scale_interval: float = 1800.0,
                 enabled: bool = False):
        super().__init__()
        self._job_resource = job_resource
        self._job_nodes = job_nodes
        self._job_optimizer = job_optimizer
        self._speed_monitor = speed_monitor
        self._worker_manager = worker_manager
        self._scaler = node_scaler
        self._scale_interval = scale_interval
        self._enabled = enabled
        self._started = False
        self._stop = threading.Event()

    def start_auto_scaling(self):
        if self._started:
            return
        self._started = True
        if self._enabled:
            threading.Thread(target=self._periodic_adjust_worker, daemon=True, name="dwamd-autoscaler").start()

    def stop_auto_scaling(self):
        self._stop.set()

    def _get_alive_worker_num(self) -> int:
        return sum(1 for n in self._job_nodes.get(NodeType.WORKER, {}).values()
                   if n.status in (NodeStatus.RUNNING, NodeStatus.PENDING, NodeStatus.INITIAL,
                                   NodeStatus.SUCCEEDED) and not n.is_released)

    def adjust_once(self) -> Optional[ScalePlan]:
        alive = self._get_alive_worker_num()
        ro = getattr(self._job_optimizer, "resource_optimizer", None)
        speed = self._speed_monitor.running_speed() if self._speed_monitor is not None else 0.0
        if ro is not None and speed > 0 and alive > 0:
            ro.report_speed(alive, speed)  # one point of the speed-vs-workers curve
        self._job_optimizer.set_alive_node_num(alive)
        plan = self._job_optimizer.get_job_resource_plan()
        g = plan.node_group_resources.get(NodeType.WORKER)
        if g is None or g.count <= alive:
            return None
        return self.execute_job_optimization_plan(plan)

    def _periodic_adjust_worker(self):
        while not self._stop.wait(self._scale_interval):
            try:
                self.adjust_once()
            except Exception as e:
                logger.warning(f"auto-scaling failed: {e}")

    def execute_job_optimization_plan(self, plan: ResourcePlan) -> ScalePlan:
        sp = ScalePlan()
        if not plan or plan.empty():
            return sp
        for node_type, group in plan.node_group_resources.items():
            if node_type != NodeType.WORKER or group.count <= 0:
                continue
            self._job_resource.update_node_group_resource(node_type, group.count, group.node_resource.cpu,
                                                          group.node_resource.memory)
            self._speed_monitor.set_target_worker_num(group.count)
            sp.merge(self._worker_manager.adjust_worker(self._job_resource.get_node_group_resource(node_type)))
        if not sp.empty():
            self._scaler.scale(sp)
        return sp


class PSTrainingAutoScaler(JobAutoScaler):
    """Parameter-server jobs (TF/PS) are out of scope on MI355X GPU
    training; kept as the interface the master instantiates for PS jobs."""

    def __init__(self, job_resource, job_nodes, job_optimizer: PSJobResourceOptimizer, node_scaler):
        super().__init__()
        self._job_resource = job_resource
        self._job_nodes = job_nodes
        self._job_optimizer = job_optimizer
        self._scaler = node_scaler

    def start_auto_scaling(self):
        pass

    def stop_auto_scaling(self):
        pass

    def execute_job_optimization_plan(self, plan: ResourcePlan) -> ScalePlan:
        sp = ScalePlan()
        for name, r in plan.node_resources.items():
            for nodes in self._job_nodes.values():
                for n in nodes.values():
                    if n.name == name:
                        n.config_resource = r
        return sp


def new_job_auto_scaler(strategy: str, job_resource: JobResource, job_nodes, speed_monitor, worker_manager,
                        node_scaler, enabled: bool = False, node_unit: int = 1, resource_optimizer=None,
                        max_workers: int = 0) -> JobAutoScaler:
    from ..common.constants import DistributionStrategy

    if strategy == DistributionStrategy.PS:
        return PSTrainingAutoScaler(job_resource, job_nodes, PSJobResourceOptimizer(job_resource), node_scaler)
    opt = AllreduceJobResourceOptimizer(job_resource, max_workers=max_workers, node_unit=node_unit,
                                        resource_optimizer=resource_optimizer)
    return AllreduceTrainingAutoScaler(job_resource, job_nodes, opt, speed_monitor, worker_manager, node_scaler,
                                       enabled=enabled)


def _now():
    return time.time()
