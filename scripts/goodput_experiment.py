"""Goodput under an injected rank failure, end to end through dwamd-run.

Launches ``dwamd-run`` on ``examples/train_gpt2_elastic.py`` with a fault
injected at ``--fail-step`` (the rank process exits), lets the agent persist
the breakpoint checkpoint, re-rendezvous, restart the workers (new
processes: HIP init, model build, in-place restore from shm) and finish.

goodput = (steps * median healthy step time) / (wall from the first step's
start to the last step's end).  Also reports the recovery gap (last step end
before the failure -> first step end after it, minus one step).
"""

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nproc", type=int, default=1)
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--fail-step", type=int, default=22)
    p.add_argument("--ckpt-interval", type=int, default=4)
    p.add_argument("--model", default="gpt2-1.5b")
    p.add_argument("--micro-batch", type=int, default=8)
    p.add_argument("--seq", type=int, default=1024)
    p.add_argument("--out", default="gpurun_out/goodput.json")
    p.add_argument("--timeout", type=int, default=900)
    a = p.parse_args()
    log = f"/tmp/dwamd_goodput_{os.getpid()}.jsonl"
    env = dict(os.environ, DWAMD_FAULT_INJECT_STEP=str(a.fail_step), DWAMD_FAULT_INJECT_RANK="0",
               DWAMD_SHM_PREFIX=f"gp{os.getpid()}", PYTHONPATH=REPO,
               DWAMD_STANDBY_DELAY=os.environ.get("DWAMD_STANDBY_DELAY", "1"))
    cmd = [sys.executable, "-m", "dlrover_wuqiong_amd.trainer.run", "--nnodes", "1", "--nproc-per-node",
           str(a.nproc), "--max-restarts", "2", os.path.join(REPO, "examples", "train_gpt2_elastic.py"),
           "--model", a.model, "--micro-batch", str(a.micro_batch), "--seq", str(a.seq), "--steps", str(a.steps),
           "--ckpt-interval", str(a.ckpt_interval), "--step-log", log]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, timeout=a.timeout)
    wall = time.time() - t0
    ev = [json.loads(x) for x in open(log)]
    os.remove(log)
    starts = [e for e in ev if e["event"] == "start"]
    steps = [e for e in ev if e["event"] == "step"]
    # healthy step durations: consecutive step ends within the same run
    durs = []
    for prev, cur in zip(steps, steps[1:]):
        if cur["step"] == prev["step"] + 1:
            durs.append(cur["t"] - prev["t"])
    med = statistics.median(durs)
    first_start = starts[0]["t"]
    last_end = steps[-1]["t"]
    span = last_end - first_start
    useful = a.steps * med
    # recovery gap around the failure
    fail_ix = next((i for i, (p0, p1) in enumerate(zip(steps, steps[1:])) if p1["step"] <= p0["step"]), None)
    gap = None
    if fail_ix is not None:
        gap = steps[fail_ix + 1]["t"] - steps[fail_ix]["t"] - med
    res = {"rc": r.returncode, "steps": a.steps, "fail_step": a.fail_step, "median_step_s": round(med, 4),
           "span_s": round(span, 3), "useful_s": round(useful, 3), "goodput_pct": round(100 * useful / span, 2),
           "recovery_gap_s": round(gap, 3) if gap is not None else None,
           "restarts": len(starts) - 1, "resumed_from_step": starts[-1]["start_step"],
           "restore_sec_after_failure": round(starts[-1]["restore_sec"], 3),
           "restart_timeline_s": {k: round(v, 3) for k, v in starts[-1].get("timeline", {}).items()},
           "process_start_to_first_step_s": round(
               next(e["t"] for e in steps if e["t"] > starts[-1]["t"]) - starts[-1]["proc_start"], 3),
           "launcher_wall_s": round(wall, 2), "model": a.model, "nproc": a.nproc,
           "ckpt_interval": a.ckpt_interval}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    return 0 if r.returncode == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
