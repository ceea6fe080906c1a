"""bench.py end to end on CPU/gloo: 2 ranks launched through dwamd-run, one
rank SIGKILLed mid-step, the agent restarts from deep standbys, the new
processes restore from shm and finish the fault window.  The JSON line must
report the requested world size and a verified restore."""

import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_real_kill(tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--model", "gpt2-tiny", "--micro-batch",
           "2", "--seq", "64", "--steps", "8", "--warmup", "2", "--fault-window", "16", "--ckpt-dir", str(tmp_path / "ckpt"), "--timeout",
           "240"]
    r = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-20000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["rccl_world"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["steps"] == 8 and res["warmup"] == 2
    assert res["load_verified"] and res["replicas_identical"]
    assert res["restarts"] == 1 and res["load_verified_after_restart"]
    assert 0 < res["goodput_pct"] < 100
    assert res["lost_steps"] >= 0 and res["recover_sec"] > 0
    assert res["persist_sec"] is not None
