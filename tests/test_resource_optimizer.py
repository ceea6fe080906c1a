"""Resource optimizer (single-job mode = the Brain algorithms over the
master's own metrics) and the Brain's PS / OOM / host-memory algorithms.
Reference: dlrover/python/tests/test_resource_optimizer.py,
test_local_optimizer.py and the Go brain optalgorithm tests."""

from dlrover_wuqiong_amd.brain.service import BrainDatastore, BrainOptimizer, MetricsType
from dlrover_wuqiong_amd.common.constants import DistributionStrategy, NodeType
from dlrover_wuqiong_amd.common.node import JobResource, NodeGroupResource, NodeResource
from dlrover_wuqiong_amd.master.resource_optimizer import (LocalResourceOptimizer, OptimizeStage, ResourceLimits,
                                                           new_resource_optimizer)


def _store(rows):
    st = BrainDatastore()
    for i, (uuid, name, user, typ, m) in enumerate(rows):
        st.persist({"job_uuid": uuid, "job_name": name, "user": user, "metrics_type": typ, "metrics": m,
                    "ts": float(i)})
    return BrainOptimizer(st, margin=0.25)


def test_ps_create_from_history_and_cold_start():
    rows = []
    for job in ("a1", "a2"):
        for ps in range(3 if job == "a1" else 4):
            rows.append((job, "ctr", "u", MetricsType.RESOURCE_USAGE,
                         {"node_type": "ps", "node_name": f"ps-{ps}", "cpu_used": 6.0, "memory_used_mb": 8000}))
    rows.append(("a1", "ctr", "u", MetricsType.JOB_META, {"model_params": 1e9}))
    opt = _store(rows)
    r = opt.optimize({"opt_type": "job_ps_create_resource", "job_uuid": "new", "job_name": "ctr"})
    assert r["ps"]["count"] == 4 and r["ps"]["memory_mb"] == 10000 and r["ps"]["cpu"] == 7.5
    # an unseen job name of the same user with a 2x model: scaled from the nearest job
    r = opt.optimize({"opt_type": "job_ps_cold_create_resource", "job_uuid": "n2", "job_name": "other",
                      "user": "u", "model_params": 1.5e9})
    assert r["source"].startswith("similar(ctr") and r["ps"]["memory_mb"] == 15000
    r = opt.optimize({"opt_type": "job_ps_create_resource", "job_uuid": "n3", "job_name": "nothing",
                      "user": "x", "model_params": 1e9})
    assert r["source"] == "default"


def test_ps_init_adjust_util_and_oom():
    rows = [("j", "n", "u", MetricsType.RESOURCE_USAGE,
             {"node_type": "ps", "node_name": "ps-0", "step": s, "memory_used_mb": 1000 + 10 * s, "cpu": 8,
              "cpu_used": 1.0}) for s in (0, 100, 200)]
    rows.append(("j", "n", "u", MetricsType.OOM, {"node_type": "ps", "memory_mb": 4000}))
    opt = _store(rows)
    r = opt.optimize({"opt_type": "job_ps_init_adjust_resource", "job_uuid": "j", "max_steps": 1000})
    assert r["ps_nodes"]["ps-0"]["memory_mb"] == int((1000 + 10 * 1000) * 1.25)
    r = opt.optimize({"opt_type": "job_ps_resource_util", "job_uuid": "j", "low_threshold": 0.3})
    assert r["ps_nodes"]["ps-0"]["cpu"] == 1.25
    assert opt.optimize({"opt_type": "job_ps_oom_resource", "job_uuid": "j"})["ps"]["memory_mb"] == 6000


def test_gpu_host_memory_for_flash_checkpoint():
    opt = _store([("j", "n", "u", MetricsType.JOB_META, {"ckpt_bytes_per_node": 8 * 22 << 30})])
    r = opt.optimize({"opt_type": "job_gpu_host_memory", "job_uuid": "j", "headroom_mb": 1024})
    assert r["worker"]["memory_mb"] == 2 * 8 * 22 * 1024 + 1024


def test_local_optimizer_stages_and_limits():
    ro = LocalResourceOptimizer("job", "llama", ResourceLimits(memory_mb=300000, max_workers=8, node_unit=2))
    plan = ro.generate_opt_plan(OptimizeStage.JOB_CREATE, {"ckpt_bytes_per_node": 176 << 30, "gpus_per_node": 8,
                                                           "workers": 5})
    w = plan.node_group_resources[NodeType.WORKER]
    assert w.count == 4 and w.node_resource.memory == 300000 and w.node_resource.gpu_num == 8
    # speed curve: near-linear to 4 nodes, flat beyond -> stay at 4
    for n, sp in ((2, 100.0), (4, 196.0), (6, 200.0)):
        ro.report_speed(n, sp)
    plan = ro.generate_opt_plan(OptimizeStage.RUNNING, {"current_workers": 6})
    assert plan.node_group_resources[NodeType.WORKER].count == 4
    # still scaling at the largest count -> one more unit, capped by max_workers
    ro2 = LocalResourceOptimizer("j2", "x", ResourceLimits(max_workers=8, node_unit=2))
    for n, sp in ((2, 100.0), (4, 199.0), (6, 297.0)):
        ro2.report_speed(n, sp)
    assert ro2.generate_opt_plan(OptimizeStage.RUNNING, {"current_workers": 6}).node_group_resources[
        NodeType.WORKER].count == 8
    oom = ro.generate_oom_recovery_plan(NodeType.WORKER, 100000)
    assert oom.node_group_resources[NodeType.WORKER].node_resource.memory == 150000


def test_ps_local_optimizer_running_plan():
    ro = new_resource_optimizer("single-job", "p", "ps-job", strategy=DistributionStrategy.PS)
    ro.report(MetricsType.RESOURCE_USAGE, {"node_type": "ps", "node_name": "ps-0", "cpu": 4, "cpu_used": 3.9})
    ro.report(MetricsType.RESOURCE_USAGE, {"node_type": "ps", "node_name": "ps-1", "cpu": 8, "cpu_used": 0.5})
    plan = ro.generate_opt_plan(OptimizeStage.RUNNING)
    assert plan.node_resources["ps-0"].cpu == 6.0 and plan.node_resources["ps-1"].cpu == 1.0


def test_autoscaler_follows_speed_curve():
    from dlrover_wuqiong_amd.common.constants import NodeStatus
    from dlrover_wuqiong_amd.master.autoscale import new_job_auto_scaler

    jr = JobResource()
    jr.node_group_resources[NodeType.WORKER] = NodeGroupResource(2, NodeResource(gpu_num=8))
    nodes = jr.init_job_node_meta(3)
    for n in nodes[NodeType.WORKER].values():
        n.status = NodeStatus.RUNNING

    class Speed:
        def running_speed(self):
            return 100.0

        def set_target_worker_num(self, n):
            self.target = n

    class WM:
        def adjust_worker(self, g):
            from dlrover_wuqiong_amd.master.scaler import ScalePlan

            return ScalePlan()

    class Sc:
        def scale(self, sp):
            pass

    ro = LocalResourceOptimizer("a", "b", ResourceLimits(max_workers=4))
    ro.report_speed(1, 52.0)
    sp = Speed()
    scaler = new_job_auto_scaler(DistributionStrategy.ALLREDUCE, jr, nodes, sp, WM(), Sc(), resource_optimizer=ro,
                                 max_workers=4)
    scaler.adjust_once()  # reports (2 workers, 100/s): still linear -> one more node
    assert sp.target == 3
