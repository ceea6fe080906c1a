"""Node event callbacks on the master.

Parity: reference ``master/node/event_callback.py`` (``NodeEventCallback``
:42, ``TaskRescheduleCallback``, ``AllReduceNodeHandlingCallback`` :218-339).
"""

import functools
import sys
from abc import ABC

from ..common.constants import JobExitReason, NodeExitReason, NodeType, RendezvousName, TrainingExceptionLevel
from ..common.log import logger
from ..common.node import Node


class NodeEventCallback(ABC):
    @staticmethod
    def log_callback_exception(func):
        @functools.wraps(func)
        def wrapper(*args, **kwargs):
            try:
                return func(*args, **kwargs)
            except Exception as e:
                logger.warning(f"node event callback {func.__name__} failed: {e}", exc_info=True)

        return wrapper

    def on_node_started(self, node: Node, cluster_context=None):
        pass

    def on_node_succeeded(self, node: Node, cluster_context=None):
        pass

    def on_node_failed(self, node: Node, cluster_context=None):
        pass

    def on_node_deleted(self, node: Node, cluster_context=None):
        pass


class TaskRescheduleCallback(NodeEventCallback):
    """Return the data shards a dead worker held to the todo queue."""

    def __init__(self, task_manager):
        self._task_manager = task_manager

    @NodeEventCallback.log_callback_exception
    def on_node_failed(self, node, cluster_context=None):
        if node.type == NodeType.WORKER:
            self._task_manager.recover_tasks(node.id)

    @NodeEventCallback.log_callback_exception
    def on_node_deleted(self, node, cluster_context=None):
        if node.type == NodeType.WORKER:
            self._task_manager.recover_tasks(node.id)


class PsClusterVersionCallback(NodeEventCallback):
    """A PS that fails or is removed changes the PS cluster: bump the global
    cluster version so workers rebuild their sessions (reference
    ``event_callback.py:186,199``)."""

    def __init__(self, elastic_ps):
        self._ps = elastic_ps

    @NodeEventCallback.log_callback_exception
    def on_node_failed(self, node, cluster_context=None):
        if node.type == NodeType.PS:
            self._ps.inc_global_cluster_version()

    @NodeEventCallback.log_callback_exception
    def on_node_deleted(self, node, cluster_context=None):
        if node.type == NodeType.PS:
            self._ps.inc_global_cluster_version()


class AllReduceNodeHandlingCallback(NodeEventCallback):
    """Keeps rendezvous membership in sync with node life-cycle and stops the
    job when a critical node fails for good or too many workers failed."""

    def __init__(self, master):
        self._master = master
        rdzv = master.rdzv_managers.get(RendezvousName.ELASTIC_TRAINING)
        self._min_node = rdzv.get_min_nodes() if rdzv else sys.maxsize
        self._failed_worker_count = 0
        self._total_worker_num = max(1, master.job_manager.get_worker_num())
        self._available_worker_num = self._total_worker_num

    def get_job_exit_reason(self, node: Node) -> str:
        if self._master.task_manager.training_started() or self._master.speed_monitor.last_step_time():
            if node.type == NodeType.WORKER:
                return JobExitReason.WORKER_OOM if node.exit_reason == NodeExitReason.OOM else \
                    JobExitReason.WORKER_ERROR
            return JobExitReason.UNKNOWN_ERROR
        return JobExitReason.CODE_ERROR

    @NodeEventCallback.log_callback_exception
    def on_node_started(self, node, cluster_context=None):
        if node.type == NodeType.WORKER and node.rank_index == 0:
            self._master.job_manager.start_auto_scaling()
        for m in self._master.rdzv_managers.values():
            m.add_alive_node(node.rank_index)

    @NodeEventCallback.log_callback_exception
    def on_node_succeeded(self, node, cluster_context=None):
        jm = self._master.job_manager
        if node.critical and jm.all_critical_node_completed():
            self._master.request_stop(True, JobExitReason.SUCCEEDED, "all critical nodes completed")
        self._master.speed_monitor.remove_running_worker(node.id)
        self._remove_node_from_rdzv(node)

    @NodeEventCallback.log_callback_exception
    def on_node_failed(self, node, cluster_context=None):
        self._failed_worker_count += 1
        self._stop_job_if_needed(node)
        if node.is_unrecoverable_failure():
            self._master.speed_monitor.set_target_worker_num(max(0, self._available_worker_num))
        if node.exit_reason == NodeExitReason.HARDWARE_ERROR:
            self._master.job_manager.handle_training_failure(node.type, node.id, error_data=node.exit_reason,
                                                             level=TrainingExceptionLevel.NODE_ERROR)
        self._remove_node_from_rdzv(node)

    @NodeEventCallback.log_callback_exception
    def on_node_deleted(self, node, cluster_context=None):
        self._stop_job_if_needed(node)
        self._remove_node_from_rdzv(node)

    def _remove_node_from_rdzv(self, node):
        for m in self._master.rdzv_managers.values():
            m.remove_alive_node(node.rank_index)

    def _stop_job_if_needed(self, node: Node):
        from ..common.global_context import Context

        stop_node = False
        if node.exit_reason == NodeExitReason.FATAL_ERROR and not Context.singleton_instance().relaunch_always:
            stop_node = True
        if node.relaunch_count >= node.max_relaunch_count:
            self._available_worker_num -= 1
            stop_node = True
        reason = self.get_job_exit_reason(node)
        max_failure_num = max(self._total_worker_num, node.max_relaunch_count) * 2
        if node.critical and stop_node:
            self._master.request_stop(False, reason, f"critical node {node.name} failed: "
                                                     f"{node.unrecoverable_failure_msg}")
        elif self._failed_worker_count >= max_failure_num:
            self._master.request_stop(False, reason, f"{self._failed_worker_count} node failures")
        elif self._available_worker_num < self._min_node:
            self._master.request_stop(False, reason, f"only {self._available_worker_num} workers can still run "
                                                     f"(< min nodes {self._min_node})")
