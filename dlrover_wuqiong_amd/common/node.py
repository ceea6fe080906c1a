"""Node / resource model shared by the master's managers, scaler and watcher.

Parity: reference ``dlrover/python/common/node.py`` (``NodeResource`` :37,
``NodeGroupResource`` :124, ``Node`` :149) and ``master/resource/job.py``
(``JobResource``).  GPU resources are AMD Instinct GPUs
(``amd.com/gpu``); an MI355X node is typically 8 GPUs x 288 GB HBM3E.
"""

import copy
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from .constants import Accelerators, NodeExitReason, NodeStatus, NodeType


@dataclass
class NodeResource:
    cpu: float = 0.0
    memory: int = 0  # MiB
    gpu_type: str = Accelerators.AMD_GPU
    gpu_num: int = 0
    priority: str = ""
    image: str = ""

    def to_resource_dict(self) -> Dict[str, object]:
        d: Dict[str, object] = {"cpu": self.cpu, "memory": f"{self.memory}Mi"}
        if self.gpu_num:
            d[self.gpu_type] = self.gpu_num
        return d

    @classmethod
    def resource_str_to_node_resource(cls, s: str) -> "NodeResource":
        """``"cpu=16,memory=65536Mi,gpu=8"`` -> NodeResource."""
        r = cls()
        for kv in filter(None, (x.strip() for x in s.split(","))):
            k, v = kv.split("=", 1)
            if k == "cpu":
                r.cpu = float(v)
            elif k == "memory":
                r.memory = int(v.rstrip("Mi").rstrip("Gi")) * (1024 if v.endswith("Gi") else 1)
            elif k in ("gpu", Accelerators.AMD_GPU):
                r.gpu_num = int(v)
        return r


@dataclass
class NodeGroupResource:
    count: int = 0
    node_resource: NodeResource = field(default_factory=NodeResource)

    def update(self, count: int = 0, cpu: float = 0.0, memory: int = 0):
        if count > 0:
            self.count = count
        if cpu > 0:
            self.node_resource.cpu = cpu
        if memory > 0:
            self.node_resource.memory = memory


@dataclass
class Node:
    type: str = NodeType.WORKER
    id: int = 0
    rank_index: int = 0
    name: str = ""
    status: str = NodeStatus.INITIAL
    host_addr: str = ""
    start_time: float = 0.0
    finish_time: float = 0.0
    heartbeat_time: float = 0.0
    relaunch_count: int = 0
    max_relaunch_count: int = 3
    relaunchable: bool = True
    exit_reason: str = ""
    critical: bool = False
    is_released: bool = False
    config_resource: NodeResource = field(default_factory=NodeResource)
    used_cpu: float = 0.0
    used_memory: int = 0
    gpu_stats: List = field(default_factory=list)
    paral_config: object = None
    restart_training: bool = False
    reported_failures: List[Tuple[str, str]] = field(default_factory=list)
    is_recovered_oom: bool = False  # relaunched with more memory after an OOM kill
    create_time: float = field(default_factory=time.time)

    def update_status(self, status: str) -> bool:
        from ..master.job_manager import get_node_state_flow

        if status == self.status:
            return False
        if get_node_state_flow(self.status, status) is None and self.status != NodeStatus.INITIAL:
            pass  # tolerated: watchers may skip intermediate phases
        self.status = status
        if status == NodeStatus.RUNNING and not self.start_time:
            self.start_time = time.time()
        if status in (NodeStatus.SUCCEEDED, NodeStatus.FAILED, NodeStatus.DELETED) and not self.finish_time:
            self.finish_time = time.time()
        return True

    def inc_relaunch_count(self):
        self.relaunch_count += 1

    def is_unrecoverable_failure(self) -> bool:
        return (self.relaunch_count >= self.max_relaunch_count or self.exit_reason == NodeExitReason.FATAL_ERROR
                or not self.relaunchable)

    @property
    def unrecoverable_failure_msg(self) -> str:
        if self.relaunch_count >= self.max_relaunch_count:
            return f"exhausted {self.max_relaunch_count} relaunches"
        if self.exit_reason == NodeExitReason.FATAL_ERROR:
            return "fatal error"
        return "not relaunchable"

    def get_relaunch_node_info(self, new_id: int) -> "Node":
        """The replacement node: same type/rank/resources, fresh status."""
        n = copy.deepcopy(self)
        n.id = new_id
        n.name = f"{self.type}-{new_id}"
        n.status = NodeStatus.INITIAL
        n.start_time = n.finish_time = n.heartbeat_time = 0.0
        n.exit_reason = ""
        n.is_released = False
        n.reported_failures = []
        n.create_time = time.time()
        return n


@dataclass
class JobResource:
    node_group_resources: Dict[str, NodeGroupResource] = field(default_factory=dict)

    def update_node_group_resource(self, node_type: str, count: int = 0, cpu: float = 0.0, memory: int = 0):
        g = self.node_group_resources.setdefault(node_type, NodeGroupResource())
        g.update(count, cpu, memory)

    def get_node_group_resource(self, node_type: str) -> Optional[NodeGroupResource]:
        return self.node_group_resources.get(node_type)

    @property
    def worker_num(self) -> int:
        g = self.node_group_resources.get(NodeType.WORKER)
        return g.count if g else 0

    def init_job_node_meta(self, relaunch_count: int = 3) -> Dict[str, Dict[int, Node]]:
        nodes: Dict[str, Dict[int, Node]] = {}
        for t, g in self.node_group_resources.items():
            nodes[t] = {i: Node(type=t, id=i, rank_index=i, name=f"{t}-{i}", max_relaunch_count=relaunch_count,
                                config_resource=copy.deepcopy(g.node_resource),
                                critical=(t in (NodeType.CHIEF, NodeType.PS)))
                        for i in range(g.count)}
        return nodes
