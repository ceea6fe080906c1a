"""dwamd-run end to end on CPU/gloo: fault injection -> agent restart ->
restore from the in-memory flash checkpoint; two simulated nodes; network
check; rank assignment (parity: reference test_elastic_training_agent.py)."""

import json
import os
import subprocess
import sys
import time

import pytest

from conftest import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLE = os.path.join(REPO, "examples", "elastic_train.py")


def _run(args, env_extra, timeout=240):
    env = dict(os.environ)
    env.update(env_extra)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    return subprocess.Popen([sys.executable, "-m", "dlrover_wuqiong_amd.trainer.run"] + args, env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def _results(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def test_assign_ranks():
    from dlrover_wuqiong_amd.elastic_agent.agent import ElasticTrainingAgent

    world = {3: 8, 0: 8, 5: 4}
    assert ElasticTrainingAgent.assign_ranks(0, world) == (0, 20, list(range(0, 8)))
    assert ElasticTrainingAgent.assign_ranks(3, world) == (1, 20, list(range(8, 16)))
    assert ElasticTrainingAgent.assign_ranks(5, world) == (2, 20, list(range(16, 20)))


def test_single_node_fault_restart_restores_from_memory(tmp_path):
    out = tmp_path / "out.jsonl"
    p = _run(["--nnodes", "1", "--nproc-per-node", "2", "--max-restarts", "2", EXAMPLE, "--steps", "16",
              "--out", str(out), "--ckpt-dir", str(tmp_path / "ck")],
             {"DWAMD_FAULT_INJECT_STEP": "6", "DWAMD_FAULT_INJECT_RANK": "1", "DWAMD_STANDBY_DELAY": "0"})
    log, _ = p.communicate(timeout=240)
    assert p.returncode == 0, log[-3000:]
    assert "2 from warm standby" in log  # the restart reused the pre-started interpreters
    res = _results(out)
    assert len(res) == 1
    assert res[0]["restart"] == 1 and res[0]["start_step"] == 6  # resumed from the in-memory step-6 checkpoint
    # the agent persisted the breakpoint checkpoint before restarting
    assert (tmp_path / "ck" / "dlrover_latest.txt").read_text() == "6"


def test_max_restarts_exhausted_fails(tmp_path):
    bad = tmp_path / "bad.py"
    bad.write_text("import sys; sys.exit(3)\n")
    p = _run(["--nnodes", "1", "--nproc-per-node", "1", "--max-restarts", "1", str(bad)], {})
    log, _ = p.communicate(timeout=120)
    assert p.returncode == 1, log[-2000:]
    assert "max restarts" in log or "worker failure" in log


def test_two_nodes_one_fails(tmp_path):
    port = free_port()
    out = tmp_path / "out.jsonl"

    def args(node, ck):
        return ["--node-rank", str(node), "--nnodes", "2", "--nproc-per-node", "1", "--max-restarts", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(port), "--rdzv-conf", "lastcall_timeout=1",
                EXAMPLE, "--steps", "14", "--out", str(out), "--ckpt-dir", str(tmp_path / ck)]

    inject = {"DWAMD_FAULT_INJECT_STEP": "5", "DWAMD_FAULT_INJECT_RANK": "1"}
    n0 = _run(args(0, "ck0"), dict(inject, DWAMD_SHM_PREFIX=os.environ["DWAMD_SHM_PREFIX"] + "n0"))
    time.sleep(1.0)
    n1 = _run(args(1, "ck1"), dict(inject, DWAMD_SHM_PREFIX=os.environ["DWAMD_SHM_PREFIX"] + "n1"))
    try:
        l1, _ = n1.communicate(timeout=240)
        l0, _ = n0.communicate(timeout=240)
    finally:
        for p in (n0, n1):
            if p.poll() is None:
                p.kill()
    assert n0.returncode == 0, l0[-3000:]
    assert n1.returncode == 0, l1[-3000:]
    res = _results(out)
    assert res and res[-1]["world"] == 2
    # node 0's group restarts either on its own gloo failure (counted) or on
    # the membership change (not counted, torch semantics): both resume from
    # the in-memory step-5 checkpoint
    assert res[-1]["start_step"] == 5


def test_network_check_then_train(tmp_path):
    out = tmp_path / "out.jsonl"
    p = _run(["--nnodes", "1", "--nproc-per-node", "2", "--network-check", "--rdzv-conf", "lastcall_timeout=0.5",
              EXAMPLE, "--steps", "4", "--out", str(out), "--ckpt-dir", str(tmp_path / "ck")], {})
    log, _ = p.communicate(timeout=240)
    assert p.returncode == 0, log[-3000:]
    assert "network check round 0: ok=True" in log
    assert _results(out)[0]["restart"] == 0


def test_teardown_overlap_decision(monkeypatch, tmp_path):
    """Import-mode replacements start during the killed processes' teardown
    only when every GPU THIS JOB uses has room for a second copy (amdgpu
    sysfs numbers; the job's GPUs from its processes' DRM fdinfo, so another
    tenant's full GPU on a shared host does not block the overlap)."""
    from dlrover_wuqiong_amd.common.comm import GPUStats
    from dlrover_wuqiong_amd.elastic_agent import monitor
    from dlrover_wuqiong_amd.elastic_agent.agent import ElasticTrainingAgent

    seen = []

    def stats(*used):
        def f(pdevs=None):
            seen.append(pdevs)
            rows = [GPUStats(index=i, total_memory_mb=1000, used_memory_mb=u, gpu_utilization=0.0)
                    for i, u in enumerate(used)]
            return rows[:1] if pdevs else rows  # "our" GPU is card 0
        return f

    agent = ElasticTrainingAgent.__new__(ElasticTrainingAgent)
    monkeypatch.setattr(monitor.ResourceMonitor, "gpu_stats", staticmethod(stats(300, 450)))
    assert agent._teardown_overlap_ok()
    monkeypatch.setattr(monitor.ResourceMonitor, "gpu_stats", staticmethod(stats(300, 600)))
    assert not agent._teardown_overlap_ok()  # job GPUs unknown: every GPU counts
    agent._gpu_pdevs = {"0000:05:00.0"}
    assert agent._teardown_overlap_ok() and seen[-1] == {"0000:05:00.0"}
    del agent._gpu_pdevs
    monkeypatch.setattr(monitor.ResourceMonitor, "gpu_stats", staticmethod(stats()))
    assert not agent._teardown_overlap_ok()  # nothing readable: wait
    monkeypatch.setenv("DWAMD_OVERLAP_TEARDOWN_MAX_USED", "0.7")
    monkeypatch.setattr(monitor.ResourceMonitor, "gpu_stats", staticmethod(stats(600)))
    assert agent._teardown_overlap_ok()
    # a sampled worker size: room for one more worker (+ margin) decides
    monkeypatch.setenv("DWAMD_OVERLAP_TEARDOWN_MARGIN_GB", "0")
    agent._worker_vram = 300 << 20
    monkeypatch.setattr(monitor.ResourceMonitor, "gpu_stats", staticmethod(stats(650)))
    assert agent._teardown_overlap_ok()  # 350 MB free >= 300
    monkeypatch.setattr(monitor.ResourceMonitor, "gpu_stats", staticmethod(stats(750)))
    assert not agent._teardown_overlap_ok()  # 250 MB free
    # ... unless the standby that replaces the worker already holds part of it
    agent.ctl_dir = str(tmp_path)
    agent._standby = {0: None}
    (tmp_path / "standby_warm.0").write_text(f"{100 << 20}\n")
    assert agent._teardown_overlap_ok()  # needs 300 - 100 = 200 MB <= 250 free
    (tmp_path / "standby_warm.0").write_text("-1\n")  # reservation skipped
    assert not agent._teardown_overlap_ok()
    agent._standby = {}
    del agent._worker_vram
    # fdinfo parsing: drm-pdev lines of a process's open DRM fds
    fd = tmp_path / "fdinfo"
    fd.mkdir()
    (fd / "7").write_text("pos:\t0\ndrm-driver:\tamdgpu\ndrm-pdev:\t0000:75:00.0\ndrm-memory-vram:\t3 KiB\n")
    (fd / "8").write_text("pos:\t0\nflags:\t02\n")
    real_glob = monitor.glob.glob
    monkeypatch.setattr(monitor.glob, "glob", lambda pat: real_glob(str(fd / "*")) if "fdinfo" in pat
                        else real_glob(pat))
    assert monitor.ResourceMonitor.process_gpu_pdevs([1234]) == {"0000:75:00.0"}
    assert monitor.ResourceMonitor.process_gpu_usage([1234])[1] == {1234: 3 << 10}


def test_import_standby_helpers_without_gpu(monkeypatch):
    """The import standby's GPU warm-ups are no-ops (never fatal) on a host
    without a GPU; the optimizer warm-up leaves torch._dynamo imported."""
    from dlrover_wuqiong_amd.elastic_agent import standby

    monkeypatch.setenv("DWAMD_STANDBY_PRELOAD", "torch")
    standby._preload()
    assert "torch._dynamo" in sys.modules
    assert standby._gpu_init("0") is False
    assert standby._reserve_state_memory() in (0, -1)


def test_import_standby_releases_reservation_under_pressure(monkeypatch):
    """The standby's cached HBM goes back to the driver once the live
    worker's allocations push device free memory under the floor."""
    import torch

    from dlrover_wuqiong_amd.elastic_agent import standby

    freed = []
    free = {"v": 100 << 30}
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a: (free["v"], 288 << 30))
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: freed.append(1))
    assert standby._release_under_pressure(20 << 30) == 20 << 30 and not freed
    free["v"] = 10 << 30  # the worker grew: 10 GiB left < max(16 GiB, 6 % of 288)
    assert standby._release_under_pressure(20 << 30) == -1 and freed == [1]
    assert standby._release_under_pressure(-1) == -1 and freed == [1]  # released for good


def test_no_standbys_once_the_restart_budget_is_spent():
    from dlrover_wuqiong_amd.elastic_agent.agent import ElasticLaunchConfig, ElasticTrainingAgent

    ag = ElasticTrainingAgent.__new__(ElasticTrainingAgent)
    ag.config = ElasticLaunchConfig(max_nodes=1)
    ag.remaining_restarts = 1
    assert ag._standbys_useful()
    ag.remaining_restarts = 0
    assert not ag._standbys_useful()  # single node, no restart left: a standby could never run
    ag.config = ElasticLaunchConfig(max_nodes=4)
    assert ag._standbys_useful()  # membership changes still restart the workers


def test_standby_reserves_the_restart_path(monkeypatch, tmp_path):
    """Deep standby: once the live worker's warm profile (its peak) exists,
    the standby caches peak - (the model + optimizer it already built), fills
    the small-block pool once and marks the reservation; an import standby
    reserves the whole peak."""
    import torch

    from dlrover_wuqiong_amd.elastic_agent import standby, warm_profile
    from dlrover_wuqiong_amd.flash_checkpoint import hbm_tier

    GiB = 1 << 30
    calls = {"small": 0, "empty": []}
    monkeypatch.setattr(hbm_tier, "reserve_small_pool", lambda: calls.__setitem__("small", calls["small"] + 1))
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda *a: 25 * GiB)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a: (200 * GiB, 288 * GiB))
    monkeypatch.setattr(torch, "empty", lambda n, **k: calls["empty"].append(n))
    prof = {"max_reserved": 45 * GiB}
    monkeypatch.setattr(warm_profile, "load", lambda ctl, lr: prof)
    r = standby._Reservation(str(tmp_path), "0", deep=True)
    r.tick()
    r.tick()
    assert calls["small"] == 1 and calls["empty"] == [20 * GiB] and r.reserved == 20 * GiB
    assert (tmp_path / "standby_reserved.0").read_text().strip() == str(20 * GiB)
    monkeypatch.setattr(standby, "_apply_warm_profile", lambda ctl, lr: prof)
    calls["empty"].clear()
    r = standby._Reservation(str(tmp_path), "1", deep=False)
    r.tick(replay_profile=True)
    assert calls["empty"] == [45 * GiB]
