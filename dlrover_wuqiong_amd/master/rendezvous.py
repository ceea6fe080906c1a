"""Master-side rendezvous: forms the communication world of a job.

Parity: reference ``dlrover/python/master/elastic_training/rdzv_manager.py``
(``RendezvousManager`` :58-288, ``ElasticTrainingRendezvousManager``
:291-346, ``NetworkCheckRendezvousManager`` :349-565) and the topology sorter
of ``net_topology.py:57-88``.

Semantics kept from the reference:
* nodes join a waiting list; a round completes when the list reaches
  ``max_nodes``, or holds >= ``min_nodes`` and no node joined for
  ``waiting_timeout`` seconds (then truncated to a multiple of
  ``node_unit``);
* ``num_nodes_waiting`` > 0 tells running agents to restart into a new round
  (immediately if a member of the last world re-joined, else only when at
  least ``node_unit`` new nodes wait);
* network check: round 0 pairs nodes {0,1},{2,3},..; round 1 pairs the
  fastest with the slowest; a node failing both rounds is faulty; a node
  slower than 2x the median is a straggler.
"""

import math
import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Set, Tuple

from ..common.constants import NetworkFailureReason, RendezvousName
from ..common.log import logger


@dataclass
class NodeTopologyMeta:
    node_rank: int = 0
    process_num: int = 0
    node_ip: str = ""
    asw: str = ""  # access switch
    psw: str = ""  # pod switch


class DpTopologySorter:
    """Orders ranks so that nodes under the same access switch are adjacent
    (ring neighbours then share a switch)."""

    def sort(self, nodes: Dict[int, NodeTopologyMeta]) -> Dict[int, NodeTopologyMeta]:
        if not any(m.asw for m in nodes.values()):
            return dict(sorted(nodes.items()))
        by_asw: Dict[str, List[int]] = {}
        for r, m in sorted(nodes.items()):
            by_asw.setdefault(m.asw, []).append(r)
        out: Dict[int, NodeTopologyMeta] = {}
        for asw in sorted(by_asw):
            for r in by_asw[asw]:
                out[r] = nodes[r]
        return out


class RendezvousManager:
    name = ""

    def __init__(self):
        self._lock = threading.Lock()
        self._alive_nodes: Set[int] = set()
        self._waiting: Dict[int, NodeTopologyMeta] = {}
        self._world: Dict[int, NodeTopologyMeta] = {}
        self._latest_world_ranks: List[int] = []
        self._lastcall = 0.0
        self.min_nodes = 0
        self.max_nodes = 0
        self.waiting_timeout = 0.0
        self.node_unit = 1
        self._round = 0
        self._start_ts = 0.0
        self._join_times: Dict[int, float] = {}
        self._ckpt_steps: Dict[int, int] = {}
        self._sorter = DpTopologySorter()
        self.completed_rounds: List[Tuple[int, List[int], float]] = []  # (round, ranks, seconds)

    # ------------------------------------------------------------ params
    def update_rdzv_params(self, min_nodes: int, max_nodes: int, waiting_timeout: float, node_unit: int):
        with self._lock:
            if self.max_nodes == 0:
                self.min_nodes = min_nodes
                self.max_nodes = max_nodes
                self.waiting_timeout = waiting_timeout
                self.node_unit = max(1, node_unit)
                logger.info(f"{self.name} rendezvous params: min={min_nodes} max={max_nodes} "
                            f"timeout={waiting_timeout} unit={node_unit}")

    def get_min_nodes(self):
        return self.min_nodes

    def get_rdzv_round(self):
        return self._round

    # ----------------------------------------------------- alive tracking
    def add_alive_node(self, node_id: int):
        self._alive_nodes.add(node_id)

    def remove_alive_node(self, node_id: int):
        with self._lock:
            self._alive_nodes.discard(node_id)
            self._waiting.pop(node_id, None)

    def clear_waiting_nodes(self):
        with self._lock:
            self._waiting.clear()

    def not_joined_rdzv_nodes(self) -> List[int]:
        if not self._world:
            return []
        return [n for n in self._alive_nodes if n not in self._world]

    # --------------------------------------------------------------- join
    def join_rendezvous(self, node_rank: int, local_world_size: int, node_ip: str = "", asw: str = "") -> int:
        with self._lock:
            if not self._waiting:
                self._start_ts = time.time()
            if node_rank not in self._waiting:
                self._waiting[node_rank] = NodeTopologyMeta(node_rank, local_world_size, node_ip, asw)
                self._world = {}
                self._lastcall = time.time()
                self._join_times[node_rank] = round(self._lastcall - self._start_ts, 3)
            return self._round

    def _try_complete(self) -> bool:
        """Caller holds the lock."""
        n = len(self._waiting)
        if n == 0:
            return False
        take = 0
        if self.max_nodes and n >= self.max_nodes:
            take = self.max_nodes
        elif n >= max(1, self.min_nodes) and time.time() - self._lastcall >= self.waiting_timeout:
            take = n // self.node_unit * self.node_unit
        if take <= 0:
            return False
        ranks = sorted(self._waiting)[:take]
        self._world = self._sorter.sort({r: self._waiting[r] for r in ranks})
        self._latest_world_ranks = list(self._world)
        self._waiting = {r: m for r, m in self._waiting.items() if r not in self._world}
        self._lastcall = 0.0
        took = time.time() - self._start_ts if self._start_ts else 0.0
        self.completed_rounds.append((self._round, ranks, round(took, 3)))
        logger.info(f"{self.name} round {self._round} complete: nodes {ranks} in {took:.2f}s; "
                    f"join times {self._join_times}")
        self._join_times = {}
        self._start_ts = 0.0
        return True

    def num_nodes_waiting(self) -> int:
        with self._lock:
            if any(r in self._latest_world_ranks for r in self._waiting):
                return len(self._waiting)  # a member restarted -> everyone re-forms now
            if len(self._waiting) >= self.node_unit:
                return len(self._waiting)
            return 0

    def sync_ckpt_nodes(self, node_id: int, step: int) -> bool:
        """True once every node of the latest world reported the same step."""
        with self._lock:
            self._ckpt_steps[node_id] = step
            if len(set(self._ckpt_steps.values())) > 1:
                return False
            return len(self._ckpt_steps) >= len(self._latest_world_ranks)

    def get_comm_world(self, node_rank: int) -> Tuple[int, int, Dict[int, NodeTopologyMeta]]:
        raise NotImplementedError

    def report_network_check_result(self, node_id: int, normal: bool, elapsed: float):
        pass


class ElasticTrainingRendezvousManager(RendezvousManager):
    name = RendezvousName.ELASTIC_TRAINING

    def get_comm_world(self, node_rank: int):
        with self._lock:
            if not self._world:
                if self._try_complete():
                    self._round += 1
            # round number of the completed world is _round (1-based after completion)
            return self._round, 0, dict(self._world)


class NetworkCheckRendezvousManager(RendezvousManager):
    name = RendezvousName.NETWORK_CHECK
    CHECK_ROUNDS = 2

    def __init__(self):
        super().__init__()
        self._status: Dict[int, bool] = {}
        self._times: Dict[int, float] = {}
        self._reported: Set[int] = set()
        self._groups: List[Dict[int, NodeTopologyMeta]] = []
        self._fault: Set[int] = set()
        self._stragglers: Set[int] = set()

    def join_rendezvous(self, node_rank, local_world_size, node_ip="", asw=""):
        self._groups = []
        return super().join_rendezvous(node_rank, local_world_size, node_ip, asw)

    def get_comm_world(self, node_rank: int):
        with self._lock:
            if not self._groups and self._try_complete():
                self._fault.clear()
                self._stragglers.clear()
                self._groups = self._make_groups(self._round)
                if self._round % self.CHECK_ROUNDS == 0:
                    self._status.clear()
                    self._times.clear()
                self._reported = set()
                self._round += 1
                logger.info(f"network-check round {self._round}: groups {[list(g) for g in self._groups]}")
            for gi, g in enumerate(self._groups):
                if node_rank in g:
                    return self._round, gi, dict(g)
            return self._round, 0, dict(self._world)

    def _make_groups(self, rnd: int) -> List[Dict[int, NodeTopologyMeta]]:
        ranks = list(self._world)
        groups: List[Dict[int, NodeTopologyMeta]] = []
        if rnd % self.CHECK_ROUNDS == 0:
            order = ranks
            pairs = [order[i:i + 2] for i in range(0, len(order), 2)]
        else:
            # fastest with slowest (unreported/failed nodes sort last)
            order = sorted(ranks, key=lambda r: (self._times.get(r, math.inf), r))
            pairs, lo, hi = [], 0, len(order) - 1
            while lo < hi:
                pairs.append([order[lo], order[hi]])
                lo += 1
                hi -= 1
            if lo == hi:
                pairs.append([order[lo]])
        for p in pairs:
            if len(p) == 1 and groups:
                groups[-1][p[0]] = self._world[p[0]]  # odd node joins the last pair
            else:
                groups.append({r: self._world[r] for r in p})
        return groups

    def report_network_check_result(self, node_id: int, normal: bool, elapsed: float):
        with self._lock:
            self._reported.add(node_id)
            self._status[node_id] = self._status.get(node_id, False) or normal
            self._times[node_id] = round(min(self._times.get(node_id, math.inf), elapsed), 3)

    def _detect_stragglers(self) -> Dict[int, float]:
        ts = sorted(self._times.values())
        if not ts:
            return {}
        m = len(ts) // 2
        med = ts[m] if len(ts) % 2 else (ts[m] + ts[m - 1]) / 2
        return {n: t for n, t in self._times.items() if t > 2 * med}

    def check_fault_node(self) -> Tuple[List[int], str]:
        with self._lock:
            if len(self._reported) < len(self._world):
                return list(self._fault), NetworkFailureReason.WAITING_NODE
            if not self._fault:
                self._fault = {n for n, ok in self._status.items() if not ok}
                if not self._fault and not self._detect_stragglers():
                    # healthy: skip the second round next time
                    self._round = math.ceil(self._round / self.CHECK_ROUNDS) * self.CHECK_ROUNDS
            reason = NetworkFailureReason.NODE_FAILURE if self._fault else ""
            return sorted(self._fault), reason

    def get_straggler(self) -> Tuple[List[int], str]:
        with self._lock:
            if len(self._reported) < len(self._world):
                return list(self._stragglers), NetworkFailureReason.WAITING_NODE
            if not self._stragglers:
                self._stragglers = set(self._detect_stragglers())
            return sorted(self._stragglers), ""
