"""Job/node bookkeeping on the master.

Parity: reference ``dlrover/python/common/node.py`` (Node :37),
``master/node/status_flow.py:17-136`` (allowed status transitions),
``master/node/local_job_manager.py:31-175`` and the relaunch/heartbeat logic
of ``master/node/dist_job_manager.py`` (``_monitor_node_heart_beat`` :355,
``_should_relaunch`` :561, ``handle_training_failure`` :826).

Scheduling back-ends (K8s pods, Ray actors) are out of scope for this build;
``NodeLauncher`` is the seam where one plugs in: the local launcher is a
no-op because ``dwamd-run`` agents restart their own worker processes.
"""

import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

from ..common.constants import (JobConstant, NodeExitReason, NodeStatus, NodeType,
                                TrainingExceptionLevel)
from ..common.log import logger
from ..common.node import Node  # noqa: F401  (re-exported)

# (from, to) -> should_relaunch
_FLOW: Dict[Tuple[str, str], bool] = {
    (NodeStatus.INITIAL, NodeStatus.PENDING): False,
    (NodeStatus.INITIAL, NodeStatus.RUNNING): False,
    (NodeStatus.PENDING, NodeStatus.RUNNING): False,
    (NodeStatus.PENDING, NodeStatus.SUCCEEDED): False,
    (NodeStatus.PENDING, NodeStatus.FAILED): True,
    (NodeStatus.RUNNING, NodeStatus.SUCCEEDED): False,
    (NodeStatus.RUNNING, NodeStatus.FAILED): True,
    (NodeStatus.RUNNING, NodeStatus.DELETED): True,
    (NodeStatus.RUNNING, NodeStatus.BREAKDOWN): True,
    (NodeStatus.PENDING, NodeStatus.DELETED): True,
    (NodeStatus.FAILED, NodeStatus.DELETED): False,
    (NodeStatus.SUCCEEDED, NodeStatus.DELETED): False,
    (NodeStatus.INITIAL, NodeStatus.FAILED): True,
    (NodeStatus.INITIAL, NodeStatus.DELETED): False,
}


def get_node_state_flow(from_status: str, to_status: str) -> Optional[bool]:
    """None if the transition is not allowed, else whether to relaunch."""
    if from_status == to_status:
        return None
    return _FLOW.get((from_status, to_status))


class NodeLauncher:
    """Scheduler seam: (re)launch a node (pod / VM / local process group)."""

    def relaunch(self, node: Node) -> bool:
        return False

    def remove(self, node: Node):
        pass


class JobManager:
    def __init__(self, node_num: int = 1, launcher: Optional[NodeLauncher] = None,
                 heartbeat_timeout: float = JobConstant.NODE_HEARTBEAT_TIMEOUT,
                 max_relaunch_count: int = JobConstant.MAX_RESTART_DEFAULT):
        self._lock = threading.Lock()
        self.nodes: Dict[int, Node] = {}
        self.node_num = node_num
        self.launcher = launcher or NodeLauncher()
        self.heartbeat_timeout = heartbeat_timeout
        self.max_relaunch_count = max_relaunch_count
        self._stopped = False
        self.job_exit_reason = ""
        self.on_node_removed: List[Callable[[Node], None]] = []

    # ------------------------------------------------------------ nodes
    def _get(self, node_id: int, node_type: str = NodeType.WORKER) -> Node:
        n = self.nodes.get(node_id)
        if n is None:
            n = Node(type=node_type, id=node_id, rank_index=node_id, name=f"{node_type}-{node_id}",
                     max_relaunch_count=self.max_relaunch_count)
            self.nodes[node_id] = n
        return n

    def add_node(self, node_id: int, node_type: str = NodeType.WORKER, addr: str = ""):
        with self._lock:
            n = self._get(node_id, node_type)
            n.host_addr = addr or n.host_addr
            n.update_status(NodeStatus.RUNNING)
            n.heartbeat_time = time.time()
            return n

    def collect_node_heart_beat(self, node_type: str, node_id: int, timestamp: float):
        with self._lock:
            n = self._get(node_id, node_type)
            n.heartbeat_time = timestamp or time.time()
            if n.status in (NodeStatus.INITIAL, NodeStatus.PENDING):
                n.update_status(NodeStatus.RUNNING)

    def update_node_resource_usage(self, node_type: str, node_id: int, cpu: float, memory: int,
                                   gpu_stats=None):
        with self._lock:
            n = self._get(node_id, node_type)
            n.used_cpu, n.used_memory = cpu, memory
            n.gpu_stats = list(gpu_stats or [])

    def update_node_paral_config(self, node_type, node_id, paral_config):
        with self._lock:
            self._get(node_id, node_type).paral_config = paral_config

    def get_node(self, node_id: int) -> Optional[Node]:
        return self.nodes.get(node_id)

    def running_node_ids(self) -> List[int]:
        return [n.id for n in self.nodes.values() if n.status == NodeStatus.RUNNING]

    def get_running_nodes(self) -> List[Node]:
        return [n for n in self.nodes.values() if n.status == NodeStatus.RUNNING]

    # ---------------------------------------------------------- failures
    def handle_training_failure(self, node_type: str, node_id: int, restart_count: int = -1,
                                error_data: str = "", level: str = "") -> bool:
        """Returns True if the node is relaunched (node-level error)."""
        with self._lock:
            n = self._get(node_id, node_type)
            n.reported_failures.append((level, error_data[:1000]))
        if level == TrainingExceptionLevel.NODE_ERROR:
            return self._relaunch(n, NodeExitReason.HARDWARE_ERROR)
        return False

    def _should_relaunch(self, n: Node, reason: str) -> bool:
        if self._stopped:
            return False
        if reason == NodeExitReason.FATAL_ERROR:
            return False
        if n.relaunch_count >= n.max_relaunch_count:
            logger.warning(f"node {n.id} reached max relaunch count {n.max_relaunch_count}")
            return False
        return True

    def _relaunch(self, n: Node, reason: str) -> bool:
        n.exit_reason = reason
        if not self._should_relaunch(n, reason):
            return False
        n.relaunch_count += 1
        ok = self.launcher.relaunch(n)
        logger.info(f"relaunch node {n.id} ({reason}): {ok}")
        return ok

    def update_node_status(self, node_id: int, status: str, exit_reason: str = "") -> bool:
        with self._lock:
            n = self._get(node_id)
            prev = n.status
            flow = get_node_state_flow(prev, status)
            n.update_status(status)
            n.exit_reason = exit_reason or n.exit_reason
        if status in (NodeStatus.FAILED, NodeStatus.DELETED, NodeStatus.BREAKDOWN):
            for cb in self.on_node_removed:
                cb(n)
            if flow:
                self._relaunch(n, exit_reason or NodeExitReason.UNKNOWN_ERROR)
        return True

    def dead_nodes(self, now: Optional[float] = None) -> List[int]:
        now = now or time.time()
        return [n.id for n in self.nodes.values()
                if n.status == NodeStatus.RUNNING and n.heartbeat_time
                and now - n.heartbeat_time > self.heartbeat_timeout]

    def monitor_heartbeats(self, now: Optional[float] = None) -> List[int]:
        dead = self.dead_nodes(now)
        for nid in dead:
            logger.warning(f"node {nid}: no heartbeat for {self.heartbeat_timeout}s -> breakdown")
            self.update_node_status(nid, NodeStatus.BREAKDOWN, NodeExitReason.NO_HEARTBEAT)
        return dead

    # ------------------------------------------------------------ status
    def all_workers_exited(self) -> bool:
        ws = [n for n in self.nodes.values() if n.type == NodeType.WORKER]
        return bool(ws) and all(n.status in (NodeStatus.SUCCEEDED, NodeStatus.FAILED, NodeStatus.DELETED,
                                             NodeStatus.FINISHED) for n in ws)

    def all_workers_succeeded(self) -> bool:
        ws = [n for n in self.nodes.values() if n.type == NodeType.WORKER]
        return bool(ws) and all(n.status in (NodeStatus.SUCCEEDED, NodeStatus.FINISHED) for n in ws)

    def all_workers_failed(self) -> bool:
        ws = [n for n in self.nodes.values() if n.type == NodeType.WORKER]
        return bool(ws) and all(n.status == NodeStatus.FAILED for n in ws)

    def stop(self):
        self._stopped = True
