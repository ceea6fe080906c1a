"""Job master: rendezvous semantics, servicer RPCs over gRPC, data shards,
message serialisation (parity: reference python/tests/test_rdzv_manager.py,
test_servicer.py, test_master_client.py, test_task_manager.py)."""

import time

import pytest

from dlrover_wuqiong_amd.common import comm
from dlrover_wuqiong_amd.common.constants import NetworkFailureReason, NodeStatus, RendezvousName
from dlrover_wuqiong_amd.master.rendezvous import (ElasticTrainingRendezvousManager,
                                                   NetworkCheckRendezvousManager)


def test_message_roundtrip():
    m = comm.BaseRequest(node_id=3, data=comm.RendezvousState(world={0: 8, 1: 8}, round=2))
    out = comm.deserialize_message(m.serialize())
    assert out.data.world == {0: 8, 1: 8} and isinstance(out.data, comm.RendezvousState)
    kv = comm.deserialize_message(comm.KeyValuePair(key="a", value=b"\x00\xff").serialize())
    assert kv.value == b"\x00\xff"
    t = comm.deserialize_message(comm.Task(task_id=1, shard=comm.Shard(name="d", start=0, end=4)).serialize())
    assert t.shard.end == 4


def test_rdzv_completes_at_max_nodes():
    m = ElasticTrainingRendezvousManager()
    m.update_rdzv_params(2, 3, 60, 1)
    for r in (2, 0, 1):
        m.join_rendezvous(r, 8)
    rnd, _g, world = m.get_comm_world(0)
    assert rnd == 1 and list(world) == [0, 1, 2]
    assert world[0].process_num == 8


def test_rdzv_min_nodes_after_lastcall_with_node_unit():
    m = ElasticTrainingRendezvousManager()
    m.update_rdzv_params(2, 8, 0.2, 2)
    for r in range(5):
        m.join_rendezvous(r, 4)
    _, _, world = m.get_comm_world(0)
    assert world == {}  # lastcall not elapsed
    time.sleep(0.25)
    _, _, world = m.get_comm_world(0)
    assert sorted(world) == [0, 1, 2, 3]  # truncated to a multiple of node_unit
    # node 4 is still waiting but < node_unit: no restart signal
    assert m.num_nodes_waiting() == 0
    m.join_rendezvous(5, 4)
    assert m.num_nodes_waiting() == 2


def test_rdzv_member_rejoin_triggers_restart():
    m = ElasticTrainingRendezvousManager()
    m.update_rdzv_params(2, 2, 60, 4)
    m.join_rendezvous(0, 1)
    m.join_rendezvous(1, 1)
    m.get_comm_world(0)
    m.join_rendezvous(1, 1)  # a member restarted
    assert m.num_nodes_waiting() == 1


def test_sync_ckpt_nodes():
    m = ElasticTrainingRendezvousManager()
    m.update_rdzv_params(2, 2, 60, 1)
    m.join_rendezvous(0, 1)
    m.join_rendezvous(1, 1)
    m.get_comm_world(0)
    assert not m.sync_ckpt_nodes(0, 10)
    assert m.sync_ckpt_nodes(1, 10)
    assert not m.sync_ckpt_nodes(1, 11)


def test_network_check_two_rounds_find_fault_and_straggler():
    m = NetworkCheckRendezvousManager()
    m.update_rdzv_params(4, 4, 60, 1)
    for r in range(4):
        m.join_rendezvous(r, 8)
    _, g0, w0 = m.get_comm_world(0)
    _, g2, w2 = m.get_comm_world(2)
    assert sorted(w0) == [0, 1] and sorted(w2) == [2, 3] and g0 != g2
    for r, ok, t in ((0, True, 1.0), (1, False, 3600.0), (2, True, 1.1), (3, True, 5.0)):
        m.report_network_check_result(r, ok, t)
    faults, reason = m.check_fault_node()
    assert faults == [1] and reason == NetworkFailureReason.NODE_FAILURE
    stragglers, _ = m.get_straggler()
    assert stragglers == [1]  # 3600 s > 2 x median
    # round 1: everyone re-joins; fastest paired with slowest
    for r in range(4):
        m.join_rendezvous(r, 8)
    _, _, w = m.get_comm_world(0)
    assert sorted(w) == [0, 1]  # 0 fastest, 1 slowest (failed)
    _, _, w = m.get_comm_world(2)
    assert sorted(w) == [2, 3]
    # node 1 recovers in round 1 -> no fault left after both rounds
    for r, ok, t in ((0, True, 1.0), (1, True, 1.2), (2, True, 1.1), (3, True, 1.0)):
        m.report_network_check_result(r, ok, t)
    faults, reason = m.check_fault_node()
    assert faults == [] and reason == ""


def test_network_check_waits_for_reports():
    m = NetworkCheckRendezvousManager()
    m.update_rdzv_params(2, 2, 60, 1)
    m.join_rendezvous(0, 1)
    m.join_rendezvous(1, 1)
    m.get_comm_world(0)
    m.report_network_check_result(0, True, 1.0)
    _, reason = m.check_fault_node()
    assert reason == NetworkFailureReason.WAITING_NODE


@pytest.fixture()
def master():
    from dlrover_wuqiong_amd.master.master import JobMaster

    m = JobMaster(port=0, node_num=2, loop_interval=0.2)
    m.start_background()
    yield m
    m.stop()


def test_master_client_end_to_end(master):
    from dlrover_wuqiong_amd.elastic_agent.master_client import MasterClient

    c0 = MasterClient(master.addr, node_id=0, retries=2, retry_interval=0.1)
    c1 = MasterClient(master.addr, node_id=1, retries=2, retry_interval=0.1)
    c0.report_rdzv_params(2, 2, 1, 1)
    c0.join_rendezvous(0, 4)
    c1.join_rendezvous(1, 4)
    rnd, group, world = c0.get_comm_world(RendezvousName.ELASTIC_TRAINING, 0)
    assert world == {0: 4, 1: 4}
    # kv store
    c0.kv_store_set("k", b"v")
    assert c1.kv_store_get("k") == b"v"
    assert c0.kv_store_add("cnt", 2) == 2 and c1.kv_store_add("cnt", 3) == 5
    # heartbeats / nodes
    c0.report_heart_beat()
    c1.report_heart_beat()
    assert {n.id for n in c0.get_running_nodes()} == {0, 1}
    # sync
    c0.join_sync("s")
    assert not c0.sync_finished("s")
    c1.join_sync("s")
    assert c1.sync_finished("s")
    c0.barrier("b", notify=True)
    assert c1.barrier("b")
    # global step + failure report
    c0.report_global_step(5, time.time())
    c0.report_failures("boom", 0, "process_error")
    assert master.error_monitor.records[-1][2] == "boom"
    # checkpoint sync across nodes
    assert not c0.sync_checkpoint(7)
    assert c1.sync_checkpoint(7)


def test_dynamic_data_sharding(master):
    from dlrover_wuqiong_amd.elastic_agent.master_client import MasterClient

    c0 = MasterClient(master.addr, node_id=0, retries=1)
    c1 = MasterClient(master.addr, node_id=1, retries=1)
    c0.report_dataset_shard_params(batch_size=10, num_epochs=1, dataset_size=100, shuffle=False,
                                   num_minibatches_per_shard=2, dataset_name="ds")
    t0 = c0.get_task("ds")
    t1 = c1.get_task("ds")
    assert (t0.shard.start, t0.shard.end) == (0, 20) and t1.shard.start == 20
    # worker 1 dies: its shard goes back to the queue
    c1.report_node_event(NodeStatus.FAILED, "oom")
    c0.report_task_result("ds", t0.task_id)
    seen = []
    while True:
        t = c0.get_task("ds")
        if t.task_id < 0:
            break
        seen.append(t.shard.start)
        c0.report_task_result("ds", t.task_id)
    assert sorted(seen) == [20, 40, 60, 80]
    assert master.task_manager.finished()


def test_shard_checkpoint_restore():
    from dlrover_wuqiong_amd.master.shard import TaskManager

    tm = TaskManager()
    tm.new_dataset(4, 40, "d", shuffle=True, storage_type="text")
    t = tm.get_dataset_task(0, "d")
    ck = tm.get_dataset_checkpoint("d")
    tm2 = TaskManager()
    tm2.new_dataset(4, 40, "d", shuffle=True, storage_type="text")
    assert tm2.restore_dataset_from_checkpoint(ck)
    n = 0
    while tm2.get_dataset_task(0, "d") is not None:
        n += 1
    assert n == 10  # the in-flight shard is included


def test_elastic_ps_cluster_versions(master):
    """Parity: reference tests/test_elastic_ps.py + servicer cluster-version RPCs."""
    from dlrover_wuqiong_amd.common.constants import NodeType, PSClusterVersionType as V
    from dlrover_wuqiong_amd.common.node import Node
    from dlrover_wuqiong_amd.elastic_agent.master_client import MasterClient
    from dlrover_wuqiong_amd.master.event_callback import PsClusterVersionCallback

    c = MasterClient(master.addr, node_id=0, node_type=NodeType.WORKER, retries=2, retry_interval=0.1)
    assert c.get_cluster_version(V.GLOBAL, NodeType.WORKER, 0) == 0
    assert c.get_cluster_version(V.RESTORED, NodeType.WORKER, 0) == -1
    c.update_cluster_version(V.LOCAL, 3, NodeType.PS, 1)
    c.update_cluster_version(V.LOCAL, 2, NodeType.WORKER, 0)
    c.update_cluster_version(V.RESTORED, 1, NodeType.WORKER, 0)
    assert c.get_cluster_version(V.LOCAL, NodeType.PS, 1) == 3
    assert c.get_cluster_version(V.LOCAL, NodeType.WORKER, 0) == 2
    assert c.get_cluster_version(V.RESTORED, NodeType.WORKER, 0) == 1
    # a failed PS bumps the global version
    cb = PsClusterVersionCallback(master.servicer.elastic_ps)
    cb.on_node_failed(Node(NodeType.PS, 5))
    cb.on_node_failed(Node(NodeType.WORKER, 6))
    assert c.get_cluster_version(V.GLOBAL, NodeType.PS, 1) == 1
    nodes, ready, failed = c.query_ps_nodes()
    assert nodes == [] and not ready and not failed


def test_streaming_restore_resumes_offsets_not_zero():
    """A checkpointed streaming dataset resumes after the last issued offset
    (the splitter position is part of the checkpoint): after the restored
    in-flight / queued shards drain, the next shard starts where the stream
    stopped, never at 0 again."""
    from dlrover_wuqiong_amd.master.shard import TaskManager

    tm = TaskManager()
    tm.new_dataset(10, -1, "s", storage_type="stream")
    done = []
    for _ in range(20):  # consume shards up to offset 200
        t = tm.get_dataset_task(0, "s")
        done.append((t.shard.start, t.shard.end))
        tm.report_dataset_task("s", t.task_id, True)
    assert done[-1] == (190, 200)
    ck = tm.get_dataset_checkpoint("s")
    tm2 = TaskManager()
    tm2.new_dataset(10, -1, "s", storage_type="stream")
    assert tm2.restore_dataset_from_checkpoint(ck)
    starts = [tm2.get_dataset_task(0, "s").shard.start for _ in range(40)]
    assert min(starts) >= 200 and starts == sorted(starts) and len(set(starts)) == 40
    assert tm2.get_dataset("s").completed_steps == 20


def test_streaming_partitions_round_robin_and_checkpoint():
    from dlrover_wuqiong_amd.master.shard import TaskManager

    tm = TaskManager()
    tm.new_dataset(5, 60, "p", storage_type="stream", partition_offsets={"a": 100, "b": 0})
    got = []
    while True:
        t = tm.get_dataset_task(0, "p")
        if t is None:
            break
        got.append((t.shard.name, t.shard.start, t.shard.end))
        tm.report_dataset_task("p", t.task_id, True)
        if len(got) == 4:
            ck = tm.get_dataset_checkpoint("p")
    assert got[:4] == [("a", 100, 105), ("b", 0, 5), ("a", 105, 110), ("b", 5, 10)]
    assert sum(e - s for _n, s, e in got) == 60 and tm.finished()
    tm2 = TaskManager()
    tm2.new_dataset(5, 60, "p", storage_type="stream", partition_offsets={"a": 100, "b": 0})
    tm2.restore_dataset_from_checkpoint(ck)
    rest = []
    while (t := tm2.get_dataset_task(0, "p")) is not None:
        rest.append((t.shard.name, t.shard.start, t.shard.end))
        tm2.report_dataset_task("p", t.task_id, True)
    assert rest == got[4:]  # exactly the remainder, no replay


def test_poison_shard_is_dropped_after_max_retries():
    from dlrover_wuqiong_amd.master.shard import TaskManager

    tm = TaskManager()
    tm.new_dataset(10, 30, "d")
    ds = tm.get_dataset("d")
    fails = 0
    for _ in range(200):
        t = tm.get_dataset_task(0, "d")
        if t is None:
            break
        ok = t.shard.start != 10  # the shard [10, 20) always fails
        fails += not ok
        tm.report_dataset_task("d", t.task_id, ok)
    assert fails == ds.max_task_retries + 1  # first try + 3 retries, then dropped
    assert [(s.start, s.end) for s in ds.failed_shards] == [(10, 20)]
    assert tm.finished()
    # dead-worker and timeout re-queues count as retries too
    tm.new_dataset(7, 10, "e")
    for _ in range(10):
        t = tm.get_dataset_task(5, "e")
        if t is None:
            break
        tm.recover_tasks(5)
    assert tm.get_dataset("e").failed_shards and tm.get_dataset("e").finished()
    # completed steps round up (7 records, batch 7 -> 1; 10 records, batch 4 -> 3)
    tm.new_dataset(4, 10, "f", num_minibatches_per_shard=3)
    t = tm.get_dataset_task(0, "f")
    tm.report_dataset_task("f", t.task_id, True)
    assert tm.get_dataset("f").completed_steps == 3
