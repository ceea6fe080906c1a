"""Node watchers: turn platform state into node events for the job manager.

Parity: reference ``master/watcher/k8s_watcher.py`` (``PodWatcher.watch`` /
``list`` :194, ``K8sScalePlanWatcher`` :267) and ``ray_watcher.py``.  The
``ProcessWatcher`` observes the agent processes of a ``ProcessScaler``.
"""

import copy
import time
from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Iterator, List

from ..common.constants import NodeEventType, NodeExitReason, NodeStatus
from ..common.node import Node


@dataclass
class NodeEvent:
    event_type: str
    node: Node


class NodeWatcher(ABC):
    @abstractmethod
    def watch(self) -> Iterator[NodeEvent]:
        ...

    @abstractmethod
    def list(self) -> List[Node]:
        ...


def exit_reason_from_code(code: int) -> str:
    """Agent exit code -> node exit reason (K8s: container terminated state)."""
    if code == 0:
        return NodeExitReason.SUCCEEDED
    if code in (-9, 137):
        return NodeExitReason.KILLED
    if code == 2:  # agent saw a GPU/driver fault signature
        return NodeExitReason.HARDWARE_ERROR
    if code in (-15, 143):
        return NodeExitReason.KILLED
    return NodeExitReason.UNKNOWN_ERROR


class ProcessWatcher(NodeWatcher):
    def __init__(self, scaler, poll: float = 0.5):
        self.scaler = scaler
        self.poll = poll
        self._reported = set()
        self._running = set()

    def list(self) -> List[Node]:
        out = []
        with self.scaler._lock:
            items = list(self.scaler.procs.items())
        for nid, p in items:
            # a snapshot: the job manager owns the node objects and diffs against them
            n = copy.copy(self.scaler.nodes[nid])
            code = p.poll()
            if code is None:
                n.status = NodeStatus.RUNNING
            else:
                n.status = NodeStatus.SUCCEEDED if code == 0 else NodeStatus.FAILED
                n.exit_reason = exit_reason_from_code(code)
            out.append(n)
        return out

    def poll_events(self) -> List[NodeEvent]:
        events = []
        for n in self.list():
            if n.status == NodeStatus.RUNNING and n.id not in self._running:
                self._running.add(n.id)
                events.append(NodeEvent(NodeEventType.MODIFIED, n))
            elif n.status in (NodeStatus.SUCCEEDED, NodeStatus.FAILED) and n.id not in self._reported:
                self._reported.add(n.id)
                events.append(NodeEvent(NodeEventType.MODIFIED, n))
        return events

    def watch(self) -> Iterator[NodeEvent]:
        while True:
            for ev in self.poll_events():
                yield ev
            time.sleep(self.poll)
