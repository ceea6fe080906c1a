"""Job manager that owns the node life-cycle on a platform.

Watches node events (``NodeWatcher``), drives the node state machine,
fires ``NodeEventCallback``s, relaunches failed nodes through the node
managers + ``Scaler`` (same rank, new node id), tracks heartbeats and hosts
the job auto-scaler.

Parity: reference ``master/node/dist_job_manager.py:88-862``
(``DistributedJobManager``: ``start`` / ``_monitor_nodes`` :334 /
``_monitor_node_heart_beat`` :355 / ``_process_event`` :473 /
``_should_relaunch`` :561 / ``_relaunch_node`` :605 /
``handle_training_failure`` :826) and ``local_job_manager.py``.
"""

import threading
import time
from typing import Dict, List, Optional

from ..common.constants import (DistributionStrategy, JobConstant, NodeExitReason, NodeResourceLimit, NodeStatus,
                                NodeType, TrainingExceptionLevel)
from ..common.log import logger
from ..common.node import JobResource, Node
from .autoscale import new_job_auto_scaler
from .event_callback import NodeEventCallback
from .job_manager import JobManager, get_node_state_flow
from .node_managers import ChiefManager, EvaluatorManager, ParameterServerManager, WorkerManager
from .scaler import ScalePlan, Scaler
from .watcher import NodeEvent, NodeWatcher


class DistributedJobManager(JobManager):
    def __init__(self, job_resource: JobResource, scaler: Scaler, watcher: NodeWatcher,
                 max_relaunch_count: int = JobConstant.MAX_RESTART_DEFAULT,
                 heartbeat_timeout: float = JobConstant.NODE_HEARTBEAT_TIMEOUT, speed_monitor=None,
                 strategy: str = DistributionStrategy.ALLREDUCE, node_unit: int = 1, auto_worker: bool = False,
                 poll_interval: float = 0.5, resource_optimizer=None, max_workers: int = 0):
        super().__init__(job_resource.worker_num, None, heartbeat_timeout, max_relaunch_count)
        self.job_resource = job_resource
        self.job_nodes: Dict[str, Dict[int, Node]] = job_resource.init_job_node_meta(max_relaunch_count)
        self.nodes = self.job_nodes.setdefault(NodeType.WORKER, {})
        self._id_lock = threading.Lock()
        self._next_id = 1 + max((nid for ns in self.job_nodes.values() for nid in ns), default=-1)
        self.worker_manager = WorkerManager(self.nodes, self._new_node_id, max_relaunch_count)
        self.ps_manager = ParameterServerManager(self.job_nodes.setdefault(NodeType.PS, {}), self._new_node_id)
        self.chief_manager = ChiefManager(self.job_nodes.setdefault(NodeType.CHIEF, {}), self._new_node_id)
        self.evaluator_manager = EvaluatorManager(self.job_nodes.setdefault(NodeType.EVALUATOR, {}),
                                                  self._new_node_id)
        self._managers = {NodeType.WORKER: self.worker_manager, NodeType.PS: self.ps_manager,
                          NodeType.CHIEF: self.chief_manager, NodeType.EVALUATOR: self.evaluator_manager}
        self._scaler = scaler
        self._watcher = watcher
        self._callbacks: List[NodeEventCallback] = []
        self._poll = poll_interval
        self._thread: Optional[threading.Thread] = None
        from .services import SpeedMonitor

        self.speed_monitor = speed_monitor or SpeedMonitor()
        self.auto_scaler = new_job_auto_scaler(strategy, job_resource, self.job_nodes, self.speed_monitor,
                                               self.worker_manager, scaler, enabled=auto_worker,
                                               node_unit=node_unit, resource_optimizer=resource_optimizer,
                                               max_workers=max_workers)
        self.resource_optimizer = resource_optimizer

    # ----------------------------------------------------------- helpers
    def _new_node_id(self) -> int:
        with self._id_lock:
            nid = self._next_id
            self._next_id += 1
            return nid

    def add_node_event_callback(self, cb: NodeEventCallback):
        self._callbacks.append(cb)

    def get_worker_num(self) -> int:
        return self.job_resource.worker_num

    def start_auto_scaling(self):
        self.auto_scaler.start_auto_scaling()

    def apply_scale_plan(self, plan: ScalePlan) -> ScalePlan:
        """Manual scaling (a ScalePlan from the user / the K8s ScalePlan
        watcher): per-type target counts go through the node managers (new
        nodes get ids and ranks, surplus nodes are removed); explicit removals
        are passed through."""
        out = ScalePlan()
        for t, g in plan.node_group_resources.items():
            mgr = self._managers.get(t)
            if mgr is None or g.count <= 0:
                continue
            cur = self.job_resource.get_node_group_resource(t)
            res = cur.node_resource if cur is not None else g.node_resource
            if g.node_resource.memory or g.node_resource.cpu or g.node_resource.gpu_num:
                res = g.node_resource
            self.job_resource.update_node_group_resource(t, g.count, res.cpu, res.memory)
            if t == NodeType.WORKER:
                out.merge(self.worker_manager.adjust_worker(self.job_resource.get_node_group_resource(t)))
        for n in plan.remove_nodes:
            for mgr in self._managers.values():
                if n.id in getattr(mgr, "_nodes", {}):
                    out.merge(mgr.remove_node(n.id))
        if not out.empty():
            self._scaler.scale(out)
        return out

    def all_critical_node_completed(self) -> bool:
        crit = [n for ns in self.job_nodes.values() for n in ns.values() if n.critical and not n.is_released]
        return all(n.status in (NodeStatus.SUCCEEDED, NodeStatus.FINISHED) for n in crit)

    def _find(self, node_id: int) -> Optional[Node]:
        for ns in self.job_nodes.values():
            if node_id in ns:
                return ns[node_id]
        return None

    # -------------------------------------------------------------- run
    def start(self):
        plan = ScalePlan()
        for ns in self.job_nodes.values():
            for n in ns.values():
                n.update_status(NodeStatus.PENDING)
                plan.launch_nodes.append(n)
        self._scaler.start()
        self._scaler.scale(plan)
        self._thread = threading.Thread(target=self._monitor_nodes, daemon=True, name="dwamd-node-monitor")
        self._thread.start()

    def _monitor_nodes(self):
        while not self._stopped:
            try:
                for ev in self._watcher.poll_events():
                    self._process_event(ev)
                self._monitor_node_heart_beat()
            except Exception as e:
                logger.warning(f"node monitor: {e}", exc_info=True)
            time.sleep(self._poll)

    def _monitor_node_heart_beat(self):
        now = time.time()
        for n in list(self.nodes.values()):
            if (n.status == NodeStatus.RUNNING and n.heartbeat_time and not n.is_released
                    and now - n.heartbeat_time > self.heartbeat_timeout):
                logger.warning(f"{n.name}: no heartbeat for {self.heartbeat_timeout}s")
                n.exit_reason = NodeExitReason.NO_HEARTBEAT
                self._process_event(NodeEvent("MODIFIED", _status_copy(n, NodeStatus.FAILED)))
                self._scaler.scale(ScalePlan(remove_nodes=[n]))

    def _process_event(self, event: NodeEvent):
        src = event.node
        node = self._find(src.id)
        if node is None or node.is_released and src.status == NodeStatus.RUNNING:
            return
        prev = node.status
        new = src.status
        if new == prev:
            return
        should_relaunch = get_node_state_flow(prev, new)
        node.update_status(new)
        if src.exit_reason:
            node.exit_reason = src.exit_reason
        logger.info(f"{node.name}: {prev} -> {new} ({node.exit_reason or '-'})")
        for cb in self._callbacks:
            if new == NodeStatus.RUNNING:
                cb.on_node_started(node)
            elif new == NodeStatus.SUCCEEDED:
                cb.on_node_succeeded(node)
            elif new == NodeStatus.FAILED:
                cb.on_node_failed(node)
            elif new == NodeStatus.DELETED:
                cb.on_node_deleted(node)
        if new in (NodeStatus.FAILED, NodeStatus.DELETED) and should_relaunch and not node.is_released:
            if self._should_relaunch(node, node.exit_reason):
                self._relaunch_node(node)
            else:
                node.is_released = True

    def _should_relaunch(self, n: Node, reason: str) -> bool:
        from ..common.global_context import Context

        if self._stopped:
            return False
        if reason == NodeExitReason.FATAL_ERROR and not Context.singleton_instance().relaunch_always:
            return False
        if n.relaunch_count >= n.max_relaunch_count:
            logger.warning(f"{n.name} reached max relaunch count {n.max_relaunch_count}")
            return False
        if reason == NodeExitReason.OOM:
            mem = n.config_resource.memory
            if mem >= NodeResourceLimit.MAX_MEMORY:
                logger.warning(f"{n.name} was OOM-killed at {mem} MiB >= the {NodeResourceLimit.MAX_MEMORY} MiB "
                               "limit: not relaunching")
                return False
            n.is_recovered_oom = True
            self.adjust_oom_resource(n)
        return n.relaunchable

    @staticmethod
    def adjust_oom_resource(n: Node):
        """More host memory for the relaunch of an OOM-killed node: x factor,
        at most +MAX_INCREMENTAL_MEMORY, capped at MAX_MEMORY (reference
        dist_job_manager.py:561-580 + the job optimizer's adjust_oom_resource)."""
        mem = max(n.config_resource.memory, NodeResourceLimit.MIN_MEMORY)
        new = min(mem * NodeResourceLimit.INCREMENTAL_MEMORY_FACTOR, mem + NodeResourceLimit.MAX_INCREMENTAL_MEMORY,
                  NodeResourceLimit.MAX_MEMORY)
        logger.info(f"{n.name} OOM: memory {n.config_resource.memory} -> {new} MiB for the relaunch")
        n.config_resource.memory = int(new)

    def pending_timeout_nodes(self, timeout: Optional[float] = None) -> List[Node]:
        """Nodes stuck in PENDING longer than ``seconds_to_wait_pending_pod``
        (no schedulable GPU node): the master fails the job instead of
        waiting forever (reference ``_process_insufficient_node`` /
        pending-pod checks)."""
        from ..common.global_context import Context

        timeout = Context.singleton_instance().seconds_to_wait_pending_pod if timeout is None else timeout
        now = time.time()
        out = []
        for ns in self.job_nodes.values():
            for n in ns.values():
                if n.status == NodeStatus.PENDING and not n.is_released and now - n.create_time > timeout:
                    out.append(n)
        return out

    def is_job_pending_too_long(self, timeout: Optional[float] = None) -> bool:
        stuck = self.pending_timeout_nodes(timeout)
        if stuck:
            logger.error(f"nodes pending beyond the timeout: {[n.name for n in stuck]}")
        return bool(stuck)

    def _relaunch_node(self, node: Node):
        mgr = self._managers.get(node.type, self.worker_manager)
        plan = mgr.relaunch_node(node, remove_exited_node=True)
        self._scaler.scale(plan)

    def _relaunch(self, n: Node, reason: str) -> bool:  # JobManager hook (NODE_ERROR reports)
        n.exit_reason = reason
        if not self._should_relaunch(n, reason):
            return False
        self._relaunch_node(n)
        return True

    def handle_training_failure(self, node_type, node_id, restart_count=-1, error_data="", level=""):
        n = self._find(node_id)
        if n is None:
            return False
        n.reported_failures.append((level, error_data[:1000]))
        if level == TrainingExceptionLevel.NODE_ERROR:
            n.exit_reason = NodeExitReason.HARDWARE_ERROR
        return False  # the agent exits on node errors; the watcher event relaunches it

    def all_workers_exited(self) -> bool:
        return self.worker_manager.all_nodes_exited()

    def all_workers_succeeded(self) -> bool:
        ns = self.worker_manager.cur_nodes
        return bool(ns) and all(n.status == NodeStatus.SUCCEEDED for n in ns)

    def all_workers_failed(self) -> bool:
        return self.worker_manager.all_nodes_failed()

    def stop(self):
        super().stop()
        stop_all = getattr(self._scaler, "stop_all", None)
        if stop_all:
            stop_all()


def _status_copy(n: Node, status: str) -> Node:
    import copy

    c = copy.copy(n)
    c.status = status
    return c


LocalJobManager = JobManager
