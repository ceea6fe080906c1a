"""Pre-formed process groups (elastic_agent/pg_preform.py) on CPU/gloo.

* 8 ranks on one node: the standbys form the 8-rank group while parked; after
  a real SIGKILL every restarted rank adopts it (no cold init) and it works;
* membership change: node 0 runs alone (its standbys pre-form a 4-rank
  group), node 1 joins, the 8-rank world is NOT the standby set, so node 0's
  standbys drop the pre-formed group and every rank forms the world cold;
* in-process unit checks of the adoption rule (backend / world / rank).
"""

import json
import os
import subprocess
import sys
import time

from conftest import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "pg_preform_worker.py")


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    return subprocess.Popen([sys.executable, "-m", "dlrover_wuqiong_amd.trainer.run"] + args, env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def _records(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def test_eight_rank_restart_adopts_preformed_group(tmp_path):
    out = tmp_path / "out.jsonl"
    p = _run(["--nnodes", "1", "--nproc-per-node", "8", "--max-restarts", "1", "--monitor-interval", "0.05",
              WORKER, "--out", str(out), "--kill"],
             {"DWAMD_STANDBY_DELAY": "0", "DWAMD_FAILURE_STOP_TIMEOUT": "0"})
    log, _ = p.communicate(timeout=300)
    assert p.returncode == 0, log[-5000:]
    recs = _records(out)
    first = [r for r in recs if r["inc"] == 0]
    second = [r for r in recs if r["inc"] == 1]
    assert len(first) == 8 and not any(r["adopted"] for r in first)  # the first world forms cold
    assert sorted(r["rank"] for r in second) == list(range(8))
    assert all(r["adopted"] and r["world"] == 8 and r["sum"] == 36.0 for r in second), second
    assert "pre-formed process group adopted" in log


def test_deep_standby_script_with_imported_init_adopts(tmp_path):
    """A deep-standby script that bound ``init_process_group`` before parking
    (``from torch.distributed import init_process_group`` / a
    ``distributed_c10d`` module alias): all 8 restarted ranks adopt the
    pre-formed group, nothing raises "initialize the default process group
    twice", and the patch is removed afterwards."""
    out = tmp_path / "out.jsonl"
    p = _run(["--nnodes", "1", "--nproc-per-node", "8", "--max-restarts", "1", "--monitor-interval", "0.05",
              "--standby-mode", "deep", WORKER, "--out", str(out), "--kill", "--deep"],
             {"DWAMD_STANDBY_DELAY": "0", "DWAMD_FAILURE_STOP_TIMEOUT": "0"})
    log, _ = p.communicate(timeout=300)
    assert p.returncode == 0, log[-5000:]
    assert "twice" not in log
    recs = _records(out)
    second = [r for r in recs if r["inc"] == 1]
    assert sorted(r["rank"] for r in second) == list(range(8)), recs
    assert all(r["adopted"] and r["clean"] and r["sum"] == 36.0 for r in second), second


def test_membership_change_falls_back_to_cold_init(tmp_path):
    port = free_port()
    out = tmp_path / "out.jsonl"

    def args(node):
        return ["--node-rank", str(node), "--nnodes", "1:2", "--nproc-per-node", "4", "--max-restarts", "1",
                # node 1 must not complete a world of its own before node 0
                # (which polls for waiting nodes every 2 s) re-joins
                "--master-addr", "127.0.0.1", "--master-port", str(port), "--rdzv-conf", "lastcall_timeout=4",
                "--monitor-interval", "0.05", WORKER, "--out", str(out), "--first-world", "4"]

    base = {"DWAMD_STANDBY_DELAY": "0", "DWAMD_FAILURE_STOP_TIMEOUT": "1"}
    n0 = _run(args(0), dict(base, DWAMD_SHM_PREFIX=os.environ["DWAMD_SHM_PREFIX"] + "n0"))
    n1 = None
    try:
        # node 0 alone: 4 ranks, and its standbys pre-formed a 4-rank group
        deadline = time.time() + 180
        while time.time() < deadline and not all((tmp_path / f"out.jsonl.ready{r}").exists() for r in range(4)):
            assert n0.poll() is None, n0.communicate()[0][-5000:]
            time.sleep(0.1)
        assert all((tmp_path / f"out.jsonl.ready{r}").exists() for r in range(4))
        n1 = _run(args(1), dict(base, DWAMD_SHM_PREFIX=os.environ["DWAMD_SHM_PREFIX"] + "n1"))
        l1, _ = n1.communicate(timeout=240)
        l0, _ = n0.communicate(timeout=240)
    finally:
        for p in (n0, n1):
            if p is not None and p.poll() is None:
                p.kill()
    assert n0.returncode == 0, l0[-5000:]
    assert n1.returncode == 0, l1[-5000:]
    recs = _records(out)
    eight = [r for r in recs if r["world"] == 8]
    assert sorted(r["rank"] for r in eight) == list(range(8))
    # the 8-rank world is not node 0's standby set: nobody adopts, all work
    assert not any(r["adopted"] for r in eight) and all(r["sum"] == 36.0 for r in eight)


_UNIT = r"""
import datetime, os, sys
import torch, torch.distributed as dist
ORIG = [dist.init_process_group]  # (a list: module-global aliases are rebound by arm())
from dlrover_wuqiong_amd.elastic_agent import pg_preform
port = int(sys.argv[1])
store = dist.TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False)
os.environ.update(RANK="0", WORLD_SIZE="1")
# 1) formed, armed, and a compatible request adopts it
assert pg_preform.preform(f"127.0.0.1:{port}", "g1/", 0, 1, "gloo")
assert pg_preform._compatible("gloo", -1, -1) and pg_preform._compatible("cpu:gloo,cuda:nccl", 1, 0)
assert not pg_preform._compatible("nccl", -1, -1) and not pg_preform._compatible("gloo", 2, -1)
holder = type(sys)("user_mod"); holder.ipg = ORIG[0]; sys.modules["user_mod"] = holder
pg_preform.arm(True)
assert holder.ipg is not ORIG[0]  # module-global aliases are rebound to the adopting wrapper
holder.ipg("gloo", timeout=datetime.timedelta(seconds=77))
assert pg_preform.adopted() is not None and dist.is_initialized()
assert holder.ipg is ORIG[0]  # ... and restored by the call
from torch.distributed.distributed_c10d import _get_default_store
assert abs(_get_default_store().timeout.total_seconds() - 77) < 1  # the script's timeout, not the pre-form limit
assert dist.init_process_group is pg_preform._orig_init or pg_preform._orig_init is None  # patch removed
dist.destroy_process_group()
# 2) formed, then a mismatching request: destroyed, the world forms cold
pg_preform._state.clear(); pg_preform._adopted = None
assert pg_preform.preform(f"127.0.0.1:{port}", "g2/", 0, 1, "gloo")
pg_preform._state["world"] = 2  # as if formed for another world than the one requested
pg_preform.arm(True)
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port + 1))
holder.ipg("gloo", world_size=1, rank=0, store=dist.PrefixStore("cold/", store))  # through an alias too
assert holder.ipg is ORIG[0]
assert pg_preform.adopted() is None and pg_preform.preformed() is None and dist.is_initialized()
dist.destroy_process_group()
# 3) the agent says no: dropped at activation
assert pg_preform.preform(f"127.0.0.1:{port}", "g3/", 0, 1, "gloo")
pg_preform.arm(False)
assert not dist.is_initialized() and pg_preform.preformed() is None
print("OK")
"""


def test_adoption_rules_in_process():
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", _UNIT, str(free_port())], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-3000:]
