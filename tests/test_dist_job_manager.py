"""DistributedJobManager: OOM-killed nodes relaunch with more memory (up to
the limit), fatal errors do not relaunch, nodes stuck PENDING fail the job
(parity: reference dlrover/python/tests/test_job_manager.py OOM / pending
cases; dist_job_manager.py:561-605)."""

import copy
import time

from dlrover_wuqiong_amd.common.constants import NodeExitReason, NodeResourceLimit, NodeStatus, NodeType
from dlrover_wuqiong_amd.common.node import JobResource, NodeGroupResource, NodeResource
from dlrover_wuqiong_amd.master.dist_job_manager import DistributedJobManager
from dlrover_wuqiong_amd.master.scaler import Scaler
from dlrover_wuqiong_amd.master.watcher import NodeEvent, NodeWatcher


class FakeScaler(Scaler):
    def __init__(self):
        super().__init__("t")
        self.plans = []

    def scale(self, plan):
        self.plans.append(plan)


class FakeWatcher(NodeWatcher):
    def __init__(self):
        self.events = []

    def watch(self):
        return iter(())

    def list(self):
        return []

    def poll_events(self):
        ev, self.events = self.events, []
        return ev


def _manager(memory=8192, workers=2, max_relaunch=3):
    jr = JobResource()
    jr.node_group_resources[NodeType.WORKER] = NodeGroupResource(workers, NodeResource(cpu=8, memory=memory))
    return DistributedJobManager(jr, FakeScaler(), FakeWatcher(), max_relaunch_count=max_relaunch, poll_interval=0.01)


def _fail(jm, node, reason):
    n = copy.copy(node)
    n.status = NodeStatus.FAILED
    n.exit_reason = reason
    jm._process_event(NodeEvent("MODIFIED", n))


def _run(jm, node):
    n = copy.copy(node)
    n.status = NodeStatus.RUNNING
    jm._process_event(NodeEvent("MODIFIED", n))


def test_oom_relaunch_doubles_memory_until_the_limit():
    jm = _manager(memory=8192)
    w0 = jm.nodes[0]
    _run(jm, w0)
    _fail(jm, w0, NodeExitReason.OOM)
    new = jm._scaler.plans[-1].launch_nodes[0]
    assert new.rank_index == 0 and new.id != w0.id
    assert new.config_resource.memory == 16384 and w0.is_recovered_oom
    # at the ceiling: no further relaunch
    at_max = jm.nodes[new.id]
    at_max.config_resource.memory = NodeResourceLimit.MAX_MEMORY
    _run(jm, at_max)
    n_plans = len(jm._scaler.plans)
    _fail(jm, at_max, NodeExitReason.OOM)
    assert len(jm._scaler.plans) == n_plans and at_max.is_released


def test_oom_bump_is_capped_per_step():
    jm = _manager(memory=NodeResourceLimit.MAX_INCREMENTAL_MEMORY * 3)
    n = jm.nodes[1]
    before = n.config_resource.memory
    jm.adjust_oom_resource(n)
    assert n.config_resource.memory == before + NodeResourceLimit.MAX_INCREMENTAL_MEMORY


def test_fatal_error_is_not_relaunched():
    jm = _manager()
    w = jm.nodes[1]
    _run(jm, w)
    _fail(jm, w, NodeExitReason.FATAL_ERROR)
    assert not jm._scaler.plans and w.is_released


def test_pending_timeout():
    jm = _manager(workers=1)
    jm.nodes[0].status = NodeStatus.PENDING
    assert not jm.is_job_pending_too_long(timeout=60)
    jm.nodes[0].create_time = time.time() - 120
    assert jm.is_job_pending_too_long(timeout=60)
    jm.nodes[0].status = NodeStatus.RUNNING
    assert not jm.is_job_pending_too_long(timeout=60)
