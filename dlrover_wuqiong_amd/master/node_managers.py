"""Per-role node managers (worker / chief / evaluator / PS).

Parity: reference ``master/node/training_node.py:151-361``
(``TrainingNodeManager``), ``node/worker.py`` (``ChiefManager`` :32,
``EvaluatorManager`` :66, ``WorkerManager`` :102-307) and ``node/ps.py``
(``ParameterServerManager``).  They decide *which* nodes to launch / remove
and return a ``ScalePlan``; the scaler executes it.
"""

import itertools
import threading
from typing import Callable, Dict, List, Optional

from ..common.constants import NodeStatus, NodeType
from ..common.log import logger
from ..common.node import Node, NodeGroupResource
from .scaler import ScalePlan

_ALIVE = (NodeStatus.INITIAL, NodeStatus.PENDING, NodeStatus.RUNNING)
_EXITED = (NodeStatus.SUCCEEDED, NodeStatus.FAILED, NodeStatus.DELETED, NodeStatus.FINISHED)


class TrainingNodeManager:
    def __init__(self, nodes: Dict[int, Node], node_type: str, new_node_id: Optional[Callable[[], int]] = None):
        self._nodes = nodes
        self._type = node_type
        self._lock = threading.Lock()
        counter = itertools.count(max(nodes.keys(), default=-1) + 1)
        self._new_id = new_node_id or (lambda: next(counter))

    @property
    def cur_nodes(self) -> List[Node]:
        return [n for n in self._nodes.values() if not n.is_released]

    def update_nodes(self, nodes: Dict[int, Node]):
        self._nodes = nodes

    def running_nodes(self) -> List[Node]:
        return [n for n in self._nodes.values() if n.status == NodeStatus.RUNNING]

    def alive_nodes(self) -> List[Node]:
        return [n for n in self._nodes.values() if n.status in _ALIVE and not n.is_released]

    def all_nodes_exited(self) -> bool:
        ns = self.cur_nodes
        return bool(ns) and all(n.status in _EXITED for n in ns)

    def all_nodes_failed(self) -> bool:
        ns = self.cur_nodes
        return bool(ns) and all(n.status == NodeStatus.FAILED for n in ns)

    def remove_node(self, node_id: int) -> ScalePlan:
        plan = ScalePlan()
        with self._lock:
            n = self._nodes.get(node_id)
            if n is None or n.is_released:
                return plan
            n.is_released = True
            plan.remove_nodes.append(n)
        return plan

    def relaunch_node(self, node: Node, remove_exited_node: bool = False) -> ScalePlan:
        """Replacement node with the same rank (new id)."""
        plan = ScalePlan()
        with self._lock:
            new_id = self._new_id()
            node.inc_relaunch_count()
            new = node.get_relaunch_node_info(new_id)
            node.is_released = True
            self._nodes[new_id] = new
        logger.info(f"relaunch {node.name} as {new.name} (rank {new.rank_index}, relaunch "
                    f"{new.relaunch_count}/{new.max_relaunch_count})")
        plan.launch_nodes.append(new)
        if remove_exited_node:
            plan.remove_nodes.append(node)
        return plan

    def launch_nodes(self, count: int, resource: Optional[NodeGroupResource] = None,
                     max_relaunch_count: int = 3) -> ScalePlan:
        plan = ScalePlan()
        with self._lock:
            ranks = {n.rank_index for n in self.alive_nodes()}
            r = 0
            for _ in range(count):
                while r in ranks:
                    r += 1
                ranks.add(r)
                nid = self._new_id()
                n = Node(type=self._type, id=nid, rank_index=r, name=f"{self._type}-{nid}",
                         max_relaunch_count=max_relaunch_count,
                         config_resource=resource.node_resource if resource else Node().config_resource)
                self._nodes[nid] = n
                plan.launch_nodes.append(n)
        return plan


class ChiefManager(TrainingNodeManager):
    def __init__(self, nodes, new_node_id=None):
        super().__init__(nodes, NodeType.CHIEF, new_node_id)

    def is_chief_running(self) -> bool:
        return any(n.status == NodeStatus.RUNNING for n in self.cur_nodes)


class EvaluatorManager(TrainingNodeManager):
    def __init__(self, nodes, new_node_id=None):
        super().__init__(nodes, NodeType.EVALUATOR, new_node_id)


class ParameterServerManager(TrainingNodeManager):
    def __init__(self, nodes, new_node_id=None):
        super().__init__(nodes, NodeType.PS, new_node_id)

    def get_ps_addrs(self) -> List[str]:
        return [n.host_addr for n in sorted(self.alive_nodes(), key=lambda n: n.rank_index) if n.host_addr]


class WorkerManager(TrainingNodeManager):
    def __init__(self, nodes, new_node_id=None, max_relaunch_count: int = 3):
        super().__init__(nodes, NodeType.WORKER, new_node_id)
        self.max_relaunch_count = max_relaunch_count

    def adjust_worker(self, worker_resource: NodeGroupResource) -> ScalePlan:
        alive = sorted(self.alive_nodes(), key=lambda n: n.rank_index)
        want = worker_resource.count
        if want > len(alive):
            return self._scale_up_workers(want - len(alive), worker_resource)
        if want < len(alive):
            return self._scale_down_workers(len(alive) - want, alive)
        return ScalePlan()

    def _scale_up_workers(self, up_num: int, resource: NodeGroupResource) -> ScalePlan:
        logger.info(f"scale up {up_num} workers")
        return self.launch_nodes(up_num, resource, self.max_relaunch_count)

    def _scale_down_workers(self, down_num: int, running_workers: List[Node]) -> ScalePlan:
        plan = ScalePlan()
        for n in sorted(running_workers, key=lambda n: -n.rank_index)[:down_num]:
            if n.critical:
                continue
            plan.merge(self.remove_node(n.id))
        logger.info(f"scale down {len(plan.remove_nodes)} workers")
        return plan

    def delete_exited_workers(self) -> ScalePlan:
        plan = ScalePlan()
        for n in self.cur_nodes:
            if n.status in (NodeStatus.FAILED, NodeStatus.SUCCEEDED):
                plan.merge(self.remove_node(n.id))
        return plan

    def delete_running_workers(self) -> ScalePlan:
        plan = ScalePlan()
        for n in self.running_nodes():
            plan.merge(self.remove_node(n.id))
        return plan

    def remove_noncritical_worker(self, worker_id: int) -> ScalePlan:
        n = self._nodes.get(worker_id)
        if n is None or n.critical:
            return ScalePlan()
        return self.remove_node(worker_id)

    def remove_not_joined_rdzv_workers(self, worker_ranks: List[int]) -> ScalePlan:
        """Workers that never joined the rendezvous (e.g. stuck pending)."""
        plan = ScalePlan()
        for n in self.cur_nodes:
            if n.rank_index in worker_ranks:
                plan.merge(self.remove_node(n.id))
        return plan

    def has_exited_worker(self) -> bool:
        return any(n.status in (NodeStatus.FAILED, NodeStatus.SUCCEEDED, NodeStatus.DELETED)
                   for n in self.cur_nodes)

    def verify_restarting_training(self, node_id: int) -> bool:
        """True once (and only once) if the master asked this node to restart
        its training processes (e.g. after a hardware reset check)."""
        n = self._nodes.get(node_id)
        if n is None or not n.restart_training:
            return False
        n.restart_training = False
        return True
