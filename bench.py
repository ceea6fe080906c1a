#!/usr/bin/env python
"""Headline benchmark: flash-checkpoint save/load seconds for GPT2-1.5B DDP
and goodput under a real rank failure, on N MI355X GPUs of one node.

Metric (BASELINE.json): "ckpt save/load sec GPT2-1.5B; goodput% under
injected faults at 1/2/4/8 GPU".  Reference numbers (DLRover flash
checkpoint, GPT-2 xl 1.5B, 2x A100, docs/figures/ft_llm_training/
checkpoint_{save,load}_time): DDP save (paused training) 2.2 s, DDP load
(recovery in memory) 3.7 s.

Process structure (nothing here touches HIP before the workers exist):

  bench.py (launcher, never initialises the GPU)
    `-- dwamd-run --nproc-per-node N --standby-mode deep   (elastic agent + job master)
          |-- N worker processes  = bench.py in worker mode, one per GPU, RCCL world of N
          `-- N deep standbys     = bench.py in worker mode, parked in standby_point()

  Under ``torch.distributed.run --nproc-per-node N`` (how the driver runs
  N > 1) only RANK 0 launches; the other N-1 launcher processes exit at once,
  so the job still has exactly one process per GPU.

What a worker does (incarnation 0):
  1. builds GPT-2 xl (48 layers, 1600 hidden, 1.56 B params, random init)
     in bf16 with fp32 master weights + AdamW state in flat buffers, FlatDDP
     (RCCL bucketed all-reduce over xGMI);
  2. W warm-up steps (each followed by a flash save), then waits until every
     local standby is parked (one-time set-up cost, kept out of the timed
     window);
  3. TIMED: K steps, every ``--ckpt-interval``-th followed by a flash save of
     model + optimizer state (21.8 GB) to the node's shm
     (DdpCheckpointer, StorageType.MEMORY).  The save time is the training
     pause: save_checkpoint() + the GPU snapshot it enqueued.  Bracketed by
     barrier + cuda.synchronize on both sides; MAX over ranks;
  4. time-to-durable (pause + PCIe flush until every slice is in shm) and a
     DISK save persisted by the agent (native parallel pwrite) while
     training continues: persist GB/s and the step-time interference;
  5. fault window (64 steps): training continues with saves; half-way
     through a checkpoint interval (the expected loss of a failure at a
     random time), mid-step (after backward, before the optimizer step),
     the last rank SIGKILLs itself.

The agent detects the death, SIGKILLs the survivors stuck in RCCL, re-runs
the rendezvous (new master port -> a new RCCL world), and activates the
standbys.  Incarnation 1 restores model + optimizer from shm (sliced H2D +
RCCL all-gather over xGMI for N > 1) -- that restore time is ``load_sec``
-- and trains to the end of the window.  goodput = productive step time /
window wall time, where the window contains the saves, the lost (redone)
steps, detection, restart, RCCL re-formation, restore and the first step.

A second, shorter job measures the same failure under the agent's DEFAULT
``--standby-mode import`` (any unmodified script): the replacement is a
pre-imported Python that runs the script from the top -- model build, HIP
init, RCCL init -- and restores from host shm (the reference's
"recovery in-memory" semantics, no HBM tier).  That restore is
``load_sec_shm`` and is what ``load_vs_baseline`` compares with the
reference's 3.7 s; the deep-standby HBM restore is ``load_sec_hbm``.
``--rehearse-shared-device`` runs N ranks on cuda:0 over gloo (RCCL refuses
two ranks per device) to exercise the N>1 fault path on a 1-GPU box; its
JSON says ``"rehearsal": true`` and is never an N-GPU measurement.

Prints ONE JSON line (launcher = rank 0 of the driver's launch).
"""

import argparse
import json
import os
import shutil
import signal
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
REF_SAVE_SEC = 2.2  # DLRover DDP GPT-1.5B "DLRover Async Persist" (paused training time)
REF_LOAD_SEC = 3.7  # DLRover DDP GPT-1.5B "DLRover Recovery In-Memory"
REF_LOAD_SSD_SEC = 9.3  # DDP GPT-1.5B "Read SSD" (checkpoint_load_time figure)
METRIC = "ckpt save/load sec GPT2-1.5B; goodput% under injected faults at 1/2/4/8 GPU"
WORKER_ENV = "DWAMD_BENCH_WORKER"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=12)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--model", default="gpt2-1.5b")
    p.add_argument("--micro-batch", type=int, default=8)
    p.add_argument("--seq", type=int, default=1024)
    # checkpoint every 4 steps (~0.5 s at N=1): the previous flush of the
    # 21.8 GB payload (~0.4 s) has landed by the next save
    p.add_argument("--ckpt-interval", type=int, default=4)
    p.add_argument("--fault-window", type=int, default=64, help="steps in the measured fault window (~8 s)")
    p.add_argument("--ckpt-dir", default="/tmp/dwamd_bench_ckpt")
    p.add_argument("--no-fault", action="store_true")
    p.add_argument("--no-persist", action="store_true", help="skip the DISK persist measurement")
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--act-ckpt", action="store_true", help="activation checkpointing (Llama configs)")
    p.add_argument("--timeout", type=float, default=900.0)
    p.add_argument("--out-dir", default="", help="keep the run's logs here (default: a temp dir, removed)")
    p.add_argument("--no-import-fault", action="store_true",
                   help="skip the second job (failure under the default --standby-mode import)")
    p.add_argument("--import-window", type=int, default=32, help="fault-window steps of the import-mode job")
    p.add_argument("--no-import-hbm", action="store_true",
                   help="skip the third job (failure under the framework default: import standbys that own the "
                        "HBM tier); the second job always restores from host shm (reference semantics)")
    p.add_argument("--inject-slow-flush", type=float, default=0.0,
                   help="fault injection: from the fault window on, each shm flush sleeps this long after its "
                        "HBM snapshot (the kill then always lands mid-flush: HBM-only restore)")
    p.add_argument("--rehearse-shared-device", action="store_true",
                   help="N ranks share cuda:0 over gloo: rehearses the N>1 fault path on one GPU")
    p.add_argument("--no-frameworks", action="store_true",
                   help="skip the FSDP / Megatron flash-checkpoint rows (N=1, GPT2-1.5B only)")
    p.add_argument("--only-import", action="store_true", help=argparse.SUPPRESS)  # A/B: the import-mode job alone
    p.add_argument("--step-overlap", action="store_true",
                   help="run the optimizer update under the next forward (optimizers/overlap.py)")
    # worker-only
    p.add_argument("--run-dir", default="", help=argparse.SUPPRESS)
    p.add_argument("--phase", default="deep", choices=["deep", "import", "import_hbm"], help=argparse.SUPPRESS)
    return p.parse_args(argv)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# =========================================================================
# launcher (no HIP in this process)
# =========================================================================
_SCRUB = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK",
          "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
          "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE",
          "TORCHELASTIC_ERROR_FILE", "TORCH_NCCL_ASYNC_ERROR_HANDLING", "DLROVER_MASTER_ADDR", "NODE_RANK")


def _read_jsonl(path):
    out = []
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line:
                try:
                    out.append(json.loads(line))
                except ValueError:
                    pass
    return out


def _kill_after(a, s0):
    """Completed steps at the kill for a fault window starting at step s0:
    half-way through the window's 2nd checkpoint interval -- the expected
    loss of a failure at a uniformly random time (ckpt_interval / 2 completed
    steps plus the partial one are redone)."""
    return s0 + a.ckpt_interval + a.ckpt_interval // 2


def _job(a, n: int, mode: str, run_dir: str, tag: str):
    """One elastic job (agent + workers + standbys).  Returns (rc, wall, shm_prefix, ckpt_dir)."""
    os.makedirs(run_dir, exist_ok=True)
    prefix = f"bench{os.getpid()}{tag}"
    ckpt_dir = os.path.join(a.ckpt_dir, f"w{n}_{os.getpid()}{tag}")
    env = {k: v for k, v in os.environ.items() if k not in _SCRUB}
    env.update({
        WORKER_ENV: "1",
        "PYTHONPATH": REPO + os.pathsep + env.get("PYTHONPATH", ""),
        "DWAMD_SHM_PREFIX": prefix,
        "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
        "DWAMD_FAILURE_STOP_TIMEOUT": "0",  # survivors are stuck in RCCL with the dead rank
        # a save whose staging buffer is still flushing WAITS (and the wait is
        # part of the measured pause) instead of being skipped
        "DWAMD_CKPT_BUSY": "wait",
        # the framework default: the HBM snapshot copy runs on the compute
        # stream inside the pause.  The opt-in overlapped copy (side stream
        # under the next forward, fenced by the next optimizer step; only safe
        # when checkpointed tensors are written in optimizer.step alone) is
        # measured separately in the deep job (``save_sec_overlapped``)
        "DWAMD_OVERLAP_SNAPSHOT": os.environ.get("DWAMD_OVERLAP_SNAPSHOT", "0"),
    })
    if a.rehearse_shared_device:
        env["DWAMD_REHEARSE_SHARED_DEVICE"] = "1"
        env["DWAMD_STANDBY_PG_BACKEND"] = "gloo"  # the standbys pre-form what the workers will ask for

    if mode == "import":
        # the reference's restart semantics: the replacement restores from
        # host shm (the framework default -- job "import_hbm" -- also gives
        # import standbys the HBM tier)
        env["DWAMD_HBM_TIER"] = "0"
    phase = mode
    mode = "import" if mode == "import_hbm" else mode
    wargs = [os.path.abspath(__file__), "--run-dir", run_dir, "--gpus", str(n), "--steps", str(a.steps),
             "--warmup", str(a.warmup), "--model", a.model, "--micro-batch", str(a.micro_batch), "--seq",
             str(a.seq), "--ckpt-interval", str(a.ckpt_interval), "--fault-window",
             str(a.fault_window if mode == "deep" else a.import_window), "--ckpt-dir", ckpt_dir, "--lr", str(a.lr),
             "--phase", phase]
    if a.inject_slow_flush > 0 and mode == "deep":
        wargs += ["--inject-slow-flush", str(a.inject_slow_flush)]
    for flag in ("no_fault", "no_persist", "act_ckpt", "step_overlap"):
        if getattr(a, flag):
            wargs.append("--" + flag.replace("_", "-"))
    sb_mode = os.environ.get("DWAMD_BENCH_STANDBY", mode)  # A/B only ("off": no standby process)
    cmd = [sys.executable, "-u", "-m", "dlrover_wuqiong_amd.trainer.run", "--nnodes", "1", "--nproc-per-node",
           str(n), "--max-restarts", "1", "--monitor-interval", "0.05", "--standby-mode", sb_mode,
           "--standby-delay", "0", "--local-addr", "127.0.0.1", "--event-log", os.path.join(run_dir, "agent.jsonl")
           ] + wargs
    log(f"bench launcher ({mode} standby job):", " ".join(cmd))
    t0 = time.time()
    # the agent's and workers' output goes to stderr: stdout carries the one JSON line
    p = subprocess.Popen(cmd, env=env, stdout=sys.stderr, stderr=sys.stderr, start_new_session=True)
    try:
        # the extra import-mode job must not hold the run hostage
        rc = p.wait(timeout=a.timeout if mode == "deep" else min(a.timeout, 420.0))
    except subprocess.TimeoutExpired:
        log("bench: timeout; killing the job")
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
        rc = 124
    return rc, time.time() - t0, prefix, ckpt_dir


def _cleanup(prefix: str, ckpt_dir: str):
    for f in os.listdir("/dev/shm"):
        if f.startswith(f"dwamd_{prefix}"):
            try:
                os.remove(os.path.join("/dev/shm", f))
            except OSError:
                pass
    shutil.rmtree(ckpt_dir, ignore_errors=True)


def launcher(a) -> int:
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("TORCHELASTIC_RUN_ID") and rank != 0:
        return 0  # torchrun's other ranks: rank 0 launches one worker per GPU
    n = a.gpus
    lws = os.environ.get("LOCAL_WORLD_SIZE")
    if lws and int(lws) != n:
        log(f"bench: --gpus {n} but the launcher started {lws} processes; using --gpus")
    run_dir = a.out_dir or os.path.join("/tmp", f"dwamd_bench_{os.getpid()}")
    shutil.rmtree(run_dir, ignore_errors=True)
    os.makedirs(run_dir, exist_ok=True)
    res, rc = None, 1
    try:
        if a.only_import:
            rc, res = 0, {"metric": METRIC, "only_import": True}
            a.no_import_hbm, a.no_frameworks = True, True
        else:
            rc, wall, prefix, ck = _job(a, n, "deep", run_dir, "")
            try:
                res = summarize(a, run_dir, n, wall)
            finally:
                _cleanup(prefix, ck)
        jobs = []
        if res is not None and not a.no_fault and not a.no_import_fault:
            jobs.append(("import", "i", "import_mode"))
            if not a.no_import_hbm:
                jobs.append(("import_hbm", "h", "import_mode_hbm"))
        for mode, tag, key in jobs:
            idir = os.path.join(run_dir, mode)
            rc2, wall2, prefix2, ck2 = _job(a, n, mode, idir, tag)
            try:
                imp = summarize_import(a, idir, wall2, mode)
            finally:
                _cleanup(prefix2, ck2)
            res[key] = imp
            if rc2:
                # the headline (deep-job) numbers stand; an extra job's
                # failure is reported in the line, not as the run's status
                res[key + "_rc"] = rc2
            if imp is None or imp.get("load_sec") is None:
                continue
            src = imp.get("restore_source") or "unknown"
            sfx = "" if mode == "import" else "_hbm_tier"
            # keys follow where the bytes really came from
            res[("load_sec_" if mode == "import" else "load_sec_import_") + src.replace("->", "_to_")] = imp["load_sec"]
            res["recover_sec_import" + sfx] = imp.get("recover_sec")
            res["goodput_pct_import" + sfx] = imp.get("goodput_pct")
            if mode == "import" and src == "shm" and a.model == "gpt2-1.5b":
                # the reference's 3.7 s is a restarted process restoring
                # from host memory: compare the like-for-like number
                res["load_vs_baseline"] = round(imp["load_sec"] / REF_LOAD_SEC, 4)
                res["load_vs_baseline_basis"] = "load_sec_shm (restarted process, restore from host shm)"
        if res is not None and not a.no_frameworks and n == 1 and a.model.startswith("gpt2") and \
                not a.rehearse_shared_device:
            res.update(framework_rows(a, run_dir))
        if res is not None:
            res["launcher_wall_s"] = round(time.time() - T_LAUNCH, 1)
    finally:
        if not a.out_dir:
            shutil.rmtree(run_dir, ignore_errors=True)
    if res is None:
        log(f"bench: job failed (rc={rc}); no result")
        return rc or 1
    print(json.dumps(res), flush=True)
    return 0 if rc == 0 else rc


T_LAUNCH = time.time()

# reference rows for GPT-1.5B: flash save pause / in-memory load, seconds
REF_FRAMEWORK = {"fsdp": (2.9, 15.1), "megatron": (1.2, 2.1)}


def _json_tail(text: str):
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                pass
    return None


def framework_rows(a, run_dir) -> dict:
    """The reference's other GPT-1.5B rows, measured here so the driver's run
    carries them: FSDP (FSDP2 + FsdpShardCheckpointer, scripts/
    bench_fsdp_llama.py) and Megatron-LM layout (MegatronCheckpointer,
    scripts/bench_megatron_tp_shard.py at TP=1).  Each is a separate process
    on the same GPU, after the DDP jobs; a failure is reported, never fatal."""
    out = {}
    env = {k: v for k, v in os.environ.items() if k not in _SCRUB}
    env.update({"PYTHONPATH": REPO + os.pathsep + env.get("PYTHONPATH", ""),
                "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")})
    jobs = {
        "fsdp": ([sys.executable, "-u", os.path.join(REPO, "scripts", "bench_fsdp_llama.py"), "--model", a.model,
                  "--seq", str(a.seq), "--micro-batch", str(a.micro_batch), "--steps", "8", "--ckpt-interval", "4",
                  "--precision", "amp", "--act-ckpt", "on",
                  "--ckpt-dir", os.path.join(a.ckpt_dir, f"fsdp_{os.getpid()}")],
                 dict(MASTER_PORT=str(29571 + os.getpid() % 1000), DWAMD_SHM_PREFIX=f"bf{os.getpid()}")),
        "megatron": ([sys.executable, "-u", os.path.join(REPO, "scripts", "bench_megatron_tp_shard.py"), "--model",
                      "gpt2-1.5b" if a.model == "gpt2-1.5b" else "llama-tiny", "--tp", "1", "--saves", "3",
                      # GPT2-1.5B: real training steps between the saves (the state in Megatron's layout is views
                      # into the live model and optimizer); other models: stand-in GEMMs
                      *(["--train-steps", "4"] if a.model == "gpt2-1.5b" else ["--work-gemms", "2"]), "--ckpt-dir",
                      os.path.join(a.ckpt_dir, f"meg_{os.getpid()}")],
                     dict(DWAMD_SHM_PREFIX=f"bm{os.getpid()}")),
    }
    for name, (cmd, extra) in jobs.items():
        e = dict(env, **extra)
        t0 = time.time()
        try:
            r = subprocess.run(cmd, env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240,
                               start_new_session=True)
            with open(os.path.join(run_dir, f"{name}.err"), "w") as f:
                f.write(r.stderr[-20000:])
            j = _json_tail(r.stdout) if r.returncode == 0 else None
        except subprocess.TimeoutExpired:
            j, r = None, None
        prefix = extra.get("DWAMD_SHM_PREFIX", "")
        _cleanup(prefix, cmd[cmd.index("--ckpt-dir") + 1])
        if j is None:
            out[f"{name}_rc"] = r.returncode if r is not None else 124
            continue
        ref_save, ref_load = REF_FRAMEWORK[name]
        save = j.get("value")
        load = j.get("load_sec")
        ref = a.model == "gpt2-1.5b"
        out[name] = {"save_sec": save, "load_sec": load, "load_verified": j.get("load_verified"),
                     "save_vs_baseline": round(save / ref_save, 4) if (save and ref) else None,
                     "load_vs_baseline": round(load / ref_load, 4) if (load and ref) else None,
                     "ckpt_bytes": j.get("ckpt_bytes_per_rank", j.get("ckpt_bytes")),
                     "train_step_ms": j.get("train_step_ms"), "wall_s": round(time.time() - t0, 1),
                     "reference_s": {"save": ref_save, "load": ref_load}}
    return out


def summarize(a, run_dir, n, wall):
    ev = _read_jsonl(os.path.join(run_dir, "steps.jsonl"))
    agent = _read_jsonl(os.path.join(run_dir, "agent.jsonl"))
    phase0 = next((e for e in ev if e["event"] == "phase0"), None)
    if phase0 is None:
        return None
    step_sec = phase0["step_sec"]
    save_sec = phase0["save_sec_mean"]
    rehearsal = bool(phase0.get("rehearsal"))
    par = f"dp{phase0['world']}" + (" (rehearsal: ranks share cuda:0 over gloo)" if rehearsal else "")
    res = {
        "metric": METRIC,
        "value": round(save_sec, 4),
        "unit": "s",
        "n_gpus": 1 if rehearsal else phase0["world"],
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1000.0 * phase0["t_timed"] / a.steps, 2),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": round(save_sec / REF_SAVE_SEC, 4) if a.model == "gpt2-1.5b" else None,
        "dtype": phase0["dtype"],
        "data": "synthetic tokens, random-init weights",
        "config": {"model": phase0["desc"], "global_batch": a.micro_batch * phase0["world"], "seq_len": a.seq,
                   "parallelism": par},
        "rehearsal": rehearsal,
        "save_sec_mean": round(save_sec, 4),
        "save_sec_max": round(phase0["save_sec_max"], 4),
        "snapshot_mode": phase0.get("snapshot_copy"),
        # the training time one save costs, pause + anything it leaves to
        # the following steps (loop time per step - median step) x interval,
        # the closing wait for the last PCIe flush excluded
        "per_save_training_cost_ms": phase0.get("per_save_cost_ms"),
        # the opt-in overlapped snapshot copy (DWAMD_OVERLAP_SNAPSHOT=1): pause
        # and the same per-save cost, measured right after the timed loop
        "save_sec_overlapped": phase0.get("save_sec_overlapped"),
        "per_save_training_cost_ms_overlapped": phase0.get("per_save_cost_ms_overlapped"),
        "timed_saves": phase0.get("timed_saves"),
        "timed_saves_ok": phase0.get("timed_saves_ok"),
        "skipped_saves_timed": phase0.get("skipped_saves_timed"),
        "first_save_sec": round(phase0["first_save_sec"], 4) if phase0.get("first_save_sec") else None,
        "time_to_durable_sec": round(phase0["durable_sec"], 4),
        "flush_gbps": phase0.get("flush_gbps"),
        "load_sec_warm_process": round(phase0["load_sec_warm"], 4),
        "load_verified": phase0["load_ok"],
        "replicas_identical": phase0["replicas_identical"],
        "ckpt_interval_steps": a.ckpt_interval,
        "ckpt_bytes": phase0["ckpt_bytes"],
        "params": phase0["params"],
        "train_step_ms": round(1000 * step_sec, 2),
        "tokens_per_s": round(a.micro_batch * a.seq * phase0["world"] / step_sec, 1),
        "optimizer_update": phase0.get("optimizer_update"),
        "snapshot_copy": phase0.get("snapshot_copy"),
        "loss": phase0["loss"],
        "rccl_world": phase0["world"],
        # incarnation 0 forms its world cold: the cost a restart would pay
        # without the standbys' pre-formed group
        "pg_init_cold_sec": (phase0.get("pg") or {}).get("init_sec"),
        "backend": phase0.get("backend"),
        # replicated state split 1/N across the node's ranks (each snapshots
        # and restores its slice; restores meet in an all-gather)
        "ckpt_slices": phase0.get("slices"),
        "restore_gather_group": phase0.get("gather"),
        "hbm_plan": phase0.get("hbm_plan"),  # per-GPU budget preflight (flash_checkpoint/hbm_budget.py)
        "host_plan": phase0.get("host_plan"),  # node host-memory (tmpfs) plan of the checkpoint shm
        "launcher_wall_s": round(wall, 1),
    }
    persist = next((e for e in ev if e["event"] == "persisted"), None)
    if persist is not None and persist.get("persist_sec") is None:
        res["persist_sec"] = None  # not durable within DWAMD_BENCH_PERSIST_TIMEOUT_S
    elif persist is not None:
        res["persist_sec"] = round(persist["persist_sec"], 3)
        res["persist_gbps"] = round(phase0["ckpt_bytes"] / persist["persist_sec"] / 1e9, 2)
        res["persist_step_ms_during"] = persist.get("step_ms_during")
        res["persist_step_interference_pct"] = persist.get("interference_pct")
    sload = next((e for e in ev if e["event"] == "storage_load"), None)
    if sload is not None:
        # node replaced (shm gone): restore from the persisted file, page
        # cache dropped, O_DIRECT reads -- vs the reference's SSD read 9.3 s
        res["load_sec_storage"] = round(sload["sec"], 4)
        res["load_storage_vs_ref_ssd"] = round(sload["sec"] / REF_LOAD_SSD_SEC, 4) if a.model == "gpt2-1.5b" else None
        res["load_storage_verified"] = sload["ok"]
        res["load_storage_stats"] = sload.get("stats")
    fs = _fault_summary(a, ev, agent, step_sec, save_sec)
    if fs is None:
        res["goodput_pct"] = None
        res["load_sec"] = None
        return res
    res.update(fs)
    if res.get("restore_source") == "hbm":
        res["load_sec_hbm"] = res["load_sec"]
    res["load_vs_baseline"] = round(res["load_sec"] / REF_LOAD_SEC, 4) if a.model == "gpt2-1.5b" else None
    return res


def _fault_summary(a, ev, agent, step_sec, save_sec):
    done = next((e for e in ev if e["event"] == "done" and e.get("incarnation", 0) > 0), None)
    kill = next((e for e in ev if e["event"] == "kill"), None)
    inc1 = next((e for e in ev if e["event"] == "start" and e["incarnation"] > 0), None)
    if a.no_fault or done is None or kill is None or inc1 is None:
        return None
    fail = next((e for e in agent if e["event"] == "failure_detected"), None)
    started = [e for e in agent if e["event"] == "workers_started"]
    rdzv = [e for e in agent if e["event"] == "rendezvous"]
    restart = started[1] if len(started) > 1 else None
    steps1 = [e for e in ev if e["event"] == "step" and e.get("incarnation", 0) > 0]
    fstart = next(e for e in ev if e["event"] == "fault_start")
    window = done["t"] - fstart["t"]
    productive_steps = done["step"] - fstart["s0"]
    goodput = 100.0 * productive_steps * step_sec / window
    first_step_end = steps1[0]["t"] if steps1 else done["t"]
    # wall from the kill until the first post-restore step completes, minus
    # that step's own compute: the time with no forward progress
    recovery = first_step_end - kill["t"] - step_sec
    skipped = [e for e in ev if e["event"] == "window_skipped"]
    late = next((e for e in ev if e["event"] == "restore_late" and e.get("resident_sec") is not None), None)
    load_sec = inc1["restore_sec"] if inc1.get("restore_sec") is not None else (late or {}).get("resident_sec")
    load_ok = inc1["restore_ok"] if inc1.get("restore_ok") is not None else (late or {}).get("restore_ok")
    out = {
        "load_sec": round(load_sec, 4) if load_sec is not None else None,
        "load_verified_after_restart": load_ok,
        "load_blocking_sec": inc1.get("restore_blocking_sec"),
        "optim_restore_deferred": late is not None,
        "goodput_pct": round(goodput, 2),
        "goodput_window_s": round(window, 3),
        "goodput_window_steps": productive_steps,
        "recover_sec": round(recovery, 3),
        "lost_steps": kill["completed_step"] - inc1["restored_step"],
        "skipped_saves_fault_window": sum(e["n"] for e in skipped),
        "recovery_breakdown_s": {
            "detect": round(fail["t"] - kill["t"], 3) if fail else None,
            "agent_restart": round(restart["t"] - fail["t"], 3) if (restart and fail) else None,
            "rendezvous": rdzv[-1].get("seconds") if len(rdzv) > 1 else None,
            # import mode only (a deep standby built its model long before)
            "process_to_model_built": (round(inc1["t_model"] - inc1["t_proc"], 3)
                                       if inc1.get("standby") == "import" else None),
            "model_build_marks": inc1.get("build_marks") if inc1.get("standby") == "import" else None,
            "activate_to_pg_ready": round(inc1["t_pg"] - inc1["t_activated"], 3),
            # init_process_group + first all-reduce of the restarted world
            # (adopted: the standbys formed it while parked)
            "pg_init": (inc1.get("pg") or {}).get("init_sec"),
            "ckpt_engine_init": round(inc1["t_ckpt"] - inc1["t_pg"], 3),
            "restore": round(inc1["restore_blocking_sec"] if late is not None else inc1["restore_sec"], 3),
            "first_step": round(first_step_end - inc1["t_restored"], 3),
        },
        "pg_adopted_after_restart": (inc1.get("pg") or {}).get("adopted"),
        "pg_preform_sec": (inc1.get("pg") or {}).get("preform_sec"),
        "standby_prepin_s": inc1.get("prepin_s"),
        "restore_source": inc1.get("restore_source"),
        "restore_gather": inc1.get("restore_gather"),
        "restore_phases_s": inc1.get("restore_phases"),
        "restarts": len(started) - 1,
        # after the restart: every save's pause and the last flushes (HBM
        # staging -> shm) -- a save waits when its buffer's flush lags
        "save_ms_after_restart": [e["save_ms"] for e in steps1 if e.get("save_ms") is not None],
        "flushes_after_restart": done.get("flushes"),
        "gc_pauses_after_restart": done.get("gc_pauses"),
        # device allocations of the caching allocator from activation to the
        # 4th save after the restart (0: everything came from what the standby
        # reserved while parked)
        "device_allocs_after_restart": done.get("device_allocs_after_restart"),
    }
    # a MODEL, not a measurement: one failure per hour, a checkpoint every
    # ckpt_interval steps (mean loss: half an interval of steps)
    per_step = step_sec + save_sec / a.ckpt_interval
    fail_cost = recovery + 0.5 * a.ckpt_interval * step_sec
    out["goodput_pct_1fail_per_hour_modelled"] = round(100.0 * ((3600.0 - fail_cost) / per_step) * step_sec / 3600.0,
                                                       3)
    return out


def summarize_import(a, run_dir, wall, mode="import"):
    """The failure under the agent's default ``--standby-mode import``: the
    replacement runs the script from the top and restores from host shm
    (``import``) or from its own HBM-tier buffers (``import_hbm``)."""
    ev = _read_jsonl(os.path.join(run_dir, "steps.jsonl"))
    agent = _read_jsonl(os.path.join(run_dir, "agent.jsonl"))
    phase0 = next((e for e in ev if e["event"] == "phase0"), None)
    if phase0 is None:
        return None
    out = {"standby_mode": "import", "hbm_tier": mode == "import_hbm", "train_step_ms": round(1000 * phase0["step_sec"], 2),
           "first_save_sec": round(phase0["first_save_sec"], 4) if phase0.get("first_save_sec") else None,
           "launcher_wall_s": round(wall, 1)}
    fs = _fault_summary(a, ev, agent, phase0["step_sec"], phase0.get("save_sec_mean", 0.0))
    if fs is not None:
        out.update(fs)
    return out


# =========================================================================
# worker (one per GPU, started by the agent; also the deep standby)
# =========================================================================
def worker(a) -> int:
    t_proc = time.time()
    if os.environ.get("DWAMD_BENCH_STACK_DUMP_S"):  # hang diagnosis: every thread's stack, periodically
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["DWAMD_BENCH_STACK_DUMP_S"]), repeat=True)
    import torch
    import torch.distributed as dist

    from dlrover_wuqiong_amd.trainer.elastic import standby_point, training_stream

    lr = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    rehearsal = os.environ.get("DWAMD_REHEARSE_SHARED_DEVICE") == "1"
    # rehearsal: every rank on cuda:0 (RCCL refuses two ranks per device, so gloo)
    device = torch.device("cuda", 0 if rehearsal else lr) if cuda else torch.device("cpu")
    backend = "nccl" if (cuda and not rehearsal) else "gloo"
    backend = os.environ.get("DWAMD_BENCH_PG_BACKEND", backend)  # A/B only
    cdev = device if backend == "nccl" else torch.device("cpu")  # small control tensors
    if cuda:
        torch.cuda.set_device(device)
        # train on a dedicated non-blocking stream (not the legacy null stream);
        # an import standby's (its HBM reservation is cached for that stream)
        torch.cuda.set_stream(training_stream(device))

    from dlrover_wuqiong_amd.common.constants import CheckpointConstant
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.ddp import FlatDDP
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    from dlrover_wuqiong_amd.flash_checkpoint.deferred_init import deferred_init

    dtype = torch.bfloat16 if cuda else torch.float32
    marks = {"imports": time.time()}  # model-build phases (import-mode restarts build the model cold)
    torch.manual_seed(1234)
    # a restarted process restores every parameter: its random init is only
    # recorded (replayed if nothing was restored)
    defer = deferred_init()
    di = defer.__enter__()
    if a.model.startswith("llama") or a.model.startswith("mixtral"):
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig

        cfg = LlamaConfig.named(a.model)
        cfg.activation_checkpointing = a.act_ckpt
        with torch.device(device):
            model = Llama(cfg)
        desc = (f"{a.model} ({cfg.num_hidden_layers}L, {cfg.hidden_size}H, {cfg.num_attention_heads}/"
                f"{cfg.num_key_value_heads} heads)")
    else:
        from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

        cfg = GPT2Config.named(a.model)
        cfg.n_positions = max(cfg.n_positions, a.seq)
        with torch.device(device):
            model = GPT2(cfg)
        desc = ("GPT2-1.5B (gpt2-xl: 48L, 1600H, 25 heads)" if a.model == "gpt2-1.5b" else
                f"{a.model} ({cfg.n_layer}L, {cfg.n_embd}H, {cfg.n_head} heads)")
    defer.__exit__(None, None, None)
    if cuda:
        torch.cuda.synchronize()
    marks["init"] = time.time()
    model.to(dtype)
    nparams = model.num_params()
    flat = FlatParams(model, dtype=dtype, device=device, lazy_zero_grad=True)
    if cuda:
        torch.cuda.synchronize()
    marks["flat"] = time.time()
    opt = FusedAdamW(flat, lr=a.lr, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0)
    if cuda and a.step_overlap:
        # the update runs under the next forward (optimizers/overlap.py); the
        # timed region's closing device-wide synchronize includes all of it.
        # Off by default: +0.2 % on this step (114.83 -> 114.61 ms,
        # profiles/r4/step_ab.jsonl) -- GEMM workgroups leave no room beside
        # them -- and its side stream shares one of the 4 hardware queues
        # with the checkpoint flush, so a forward could wait behind a D2H chunk
        opt.overlap_with_forward(model)
    B, S = a.micro_batch, a.seq
    if cuda:
        torch.cuda.synchronize()
    t_model = time.time()

    from dlrover_wuqiong_amd.elastic_agent.standby import is_standby

    if is_standby():
        # load every kernel / library handle the first real step will use
        # (forward + backward, no optimizer update).  A replacement standby is
        # spawned while training runs on the same GPU, so its warm-up steals
        # GPU time from the live job: one sample (1/B of a step's FLOPs) loads
        # the same kernels; the allocator pool is released below anyway.
        wb = int(os.environ.get("DWAMD_STANDBY_WARMUP_BATCH", "1")) or B
        x = torch.randint(0, cfg.vocab_size, (min(wb, B), S + 1), device=device)
        model(x[:, :-1], x[:, 1:]).backward()
        flat.zero_grad()
        del x
        if cuda:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()  # the parked standby keeps only model + optimizer (+ HBM staging)
    def dev_allocs() -> int:
        """Device allocations the caching allocator made so far (cumulative)."""
        if not cuda:
            return 0
        st = torch.cuda.memory_stats(device)
        return int(st.get("num_device_alloc", st.get("segment.all.allocated", 0)))

    alloc0 = dev_allocs()  # import standby: this process became the worker just now
    info = standby_point()  # deep standby: parks here until the agent activates it
    t_act = time.time() if info is not None else t_proc
    if info is not None:
        alloc0 = dev_allocs()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    incarnation = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    from dlrover_wuqiong_amd.elastic_agent import pg_preform

    # a real RCCL world at every N (world 1 included): eager communicator
    # init on this GPU.  A restarted standby whose set pre-formed the world
    # while parked adopts it here (elastic_agent/pg_preform.py); otherwise
    # this is the cold re-formation the recovery pays
    t_pg0 = time.time()
    pg_world1 = world > 1 or os.environ.get("DWAMD_BENCH_PG_WORLD1", "1") == "1"  # A/B switch
    lazy = os.environ.get("DWAMD_BENCH_PG_LAZY") == "1"  # A/B only: no eager communicator, no check
    if pg_world1:
        pg_preform.init_process_group(backend, device_id=device if backend == "nccl" and not lazy else None)
    assert world == a.gpus, f"world {world} != --gpus {a.gpus}"
    ddp = FlatDDP(model, flat, bucket_mb=128)
    opt.grad_scale = 1.0 / max(1, world)
    # the communicator answers (the first collective of an adopted group
    # included) before the restore: part of the measured re-formation
    t = torch.ones(1, device=device if backend == "nccl" else torch.device("cpu"))
    if pg_world1 and not lazy:
        dist.all_reduce(t)
    if cuda:
        torch.cuda.synchronize()
    assert float(t.item()) == float(world)
    if pg_world1 and world == 1 and os.environ.get("DWAMD_BENCH_PG_DESTROY") == "1":  # A/B only
        dist.destroy_process_group()
    t_pg = time.time()
    pg_info = {"adopted": pg_preform.adopted() is not None, "init_sec": round(t_pg - t_pg0, 4),
               "preform_sec": (pg_preform.adopted() or {}).get("sec"),  # paid while parked
               "backend": backend}
    g = torch.Generator(device="cpu").manual_seed(rank)
    data = torch.randint(0, cfg.vocab_size, (4, B, S + 1), generator=g).to(device)
    ckpt = DdpCheckpointer(a.ckpt_dir)
    t_ckpt = time.time()
    step_log = os.path.join(a.run_dir, "steps.jsonl")

    def emit(obj, all_ranks=False):
        if rank == 0 or all_ranks:
            with open(step_log, "a") as f:
                f.write(json.dumps(obj) + "\n")
                f.flush()
                os.fsync(f.fileno())

    def mx(x: float) -> float:
        if world > 1:
            t = torch.tensor([x], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())
        return x

    def sync_all():
        if world > 1:
            dist.barrier()
        if cuda:
            torch.cuda.synchronize()

    step = 0

    def state():
        return {"model": model.state_dict(), "optimizer": opt.state_dict(), "step": step}

    def train_step(kill_check=True):
        nonlocal step
        batch = data[step % data.shape[0]]
        loss = ddp(batch[:, :-1], batch[:, 1:])
        loss.backward()
        if kill_check:
            _maybe_kill(step)
        ddp.finish_gradient_sync()
        opt.step()
        flat.zero_grad()
        step += 1
        return loss

    kill_after = -1
    import gc

    gc_pauses = []  # Python GC pauses >= 5 ms (diagnosis of save / step outliers)
    _gc_t = [0.0]

    def _gc_cb(phase, info):
        if phase == "start":
            _gc_t[0] = time.perf_counter()
        elif _gc_t[0]:
            dt = time.perf_counter() - _gc_t[0]
            if dt >= 0.005:
                gc_pauses.append((round(time.time(), 3), info.get("generation"), round(1000 * dt, 1)))

    gc.callbacks.append(_gc_cb)

    def _maybe_kill(completed):
        # mid-step: forward + backward enqueued (gradients all-reducing), the
        # optimizer step not yet -- SIGKILL, like a crashed / OOM-killed rank
        if incarnation == 0 and completed == kill_after and rank == world - 1:
            emit({"event": "kill", "t": time.time(), "completed_step": completed, "rank": rank}, all_ranks=True)
            os.kill(os.getpid(), signal.SIGKILL)

    def state_sums():
        opt.join()
        third = opt.master if opt.master is not None else opt.exp_avg_sq
        return [float(flat.data.float().sum()), float(opt.exp_avg.sum()), float(third.sum())]

    def state_sums_behind(deferred):
        """state_sums() computed on a side stream after a deferred restore's
        optimizer-state copies (flash_checkpoint/deferred_restore.py) and
        ordered before the first optimizer update; returns a callable that
        yields the sums (call it after that update was enqueued)."""
        from dlrover_wuqiong_amd.flash_checkpoint import deferred_restore

        opt.join()
        vs = torch.cuda.Stream()
        vs.wait_stream(torch.cuda.current_stream())
        deferred.wait(vs)
        third = opt.master if opt.master is not None else opt.exp_avg_sq
        with torch.cuda.stream(vs):
            t = torch.stack([flat.data.float().sum(), opt.exp_avg.sum(), third.sum()])
        ev = vs.record_event()
        deferred_restore.add_event(ev)  # the update waits for these reads
        return lambda: (torch.cuda.current_stream().wait_event(ev), [float(x) for x in t.tolist()])[1]

    def save(st=None):
        t0 = time.perf_counter()
        ok = ckpt.save_checkpoint(step, state(), storage_type=st or StorageType.MEMORY)
        if cuda:
            torch.cuda.current_stream().synchronize()
        return time.perf_counter() - t0, ok

    def sync_step():
        if cuda:
            # compute-stream sync only: a device-wide sync would also wait for
            # the checkpoint flush running on its own stream
            torch.cuda.current_stream().synchronize()

    def wait_standbys(marks, timeout=600.0):
        ctl = os.environ.get("DWAMD_AGENT_CTL_DIR", "")
        if not ctl or a.no_fault:
            return
        deadline = time.time() + timeout
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
        while time.time() < deadline and not all(
                os.path.exists(os.path.join(ctl, m.format(i))) for i in range(lw) for m in marks):
            time.sleep(0.05)

    if incarnation == 0 and a.phase in ("import", "import_hbm"):
        # ---------------- import-standby job: warm-up, step time, then the fault window
        first_save = None
        for _ in range(a.warmup):
            train_step(False)
            sync_step()
            dt, _ok = save()
            first_save = dt if first_save is None else first_save
        ckpt.wait_latest_checkpoint()
        times = []
        for _ in range(4):
            ts = time.perf_counter()
            train_step(False)
            sync_step()
            times.append(time.perf_counter() - ts)
        step_sec = mx(statistics.median(times))
        # the pre-imported replacements are up (on a GPU: and have replayed
        # this worker's warm profile -- recorded during the warm-up)
        wait_standbys(["standby_ready.{}"])
        if cuda:
            # ... and hold the staging buffers + restart-path reservations
            wait_standbys(["standby_warm.{}", "standby_staging.{}"], timeout=90.0)
        dt, _ok = save()
        ckpt.wait_latest_checkpoint()
        sync_all()
        emit({"event": "phase0", "world": world, "step_sec": step_sec, "save_sec_mean": mx(dt),
              "first_save_sec": first_save, "backend": backend, "pg": pg_info})
        s0 = step
        emit({"event": "fault_start", "t": time.time(), "s0": s0})
        start_step = step
    elif incarnation == 0:
        # ---------------- warm-up (includes the first, set-up-paying save)
        first_save = None
        for _ in range(a.warmup):
            train_step(False)
            sync_step()
            dt, _ok = save()
            first_save = dt if first_save is None else first_save
        ckpt.wait_latest_checkpoint()
        # wait for this node's deep standbys (built concurrently with the
        # warm-up): their one-time model build must not land in the timed
        # window.  Parked + (on a GPU) this rank's shm slices registered and
        # the HBM-tier staging buffers published
        wait_standbys(["standby_ready.{}"] + (["standby_pinned.{}", "hbm_staging.{}.json", "standby_staging.{}"]
                                              if cuda else []))
        if cuda:  # ... and the standbys' restart-path reservations (activation peak, small blocks)
            wait_standbys(["standby_reserved.{}"], timeout=90.0)
        # one untimed save: the copier switches to the standby-owned staging
        # buffers (waits for in-flight flushes once)
        save()
        ckpt.wait_latest_checkpoint()
        sync_all()

        # ---------------- timed: train + flash checkpoint every ckpt_interval steps
        save_times, step_times, losses, oks = [], [], [], []
        skipped0 = ckpt.engine.skipped_saves
        sync_all()
        t_start = time.perf_counter()
        for i in range(a.steps):
            ts = time.perf_counter()
            loss = train_step(False)
            losses.append(loss.detach())
            sync_step()
            step_times.append(time.perf_counter() - ts)
            # checkpoint after the first step of every interval: the
            # background PCIe flush then overlaps the rest of the interval
            if i % a.ckpt_interval == 0:
                dt, ok = save()
                save_times.append(dt)
                oks.append(bool(ok))
        t_loop = time.perf_counter() - t_start  # every step's compute done; the last flush may still run
        sync_all()
        t_timed = mx(time.perf_counter() - t_start)
        log(f"[rank {rank}] step ms:", [round(1000 * x, 1) for x in step_times], "save ms:",
            [round(1000 * x, 1) for x in save_times], "ok:", oks)
        # every timed save must have produced a checkpoint (a skipped save
        # would report ~0 s of pause for work that never happened)
        timed_ok = bool(mx(0.0 if all(oks) else 1.0) == 0.0)
        skipped_timed = int(mx(float(ckpt.engine.skipped_saves - skipped0)))
        ok_times = [t for t, o in zip(save_times, oks) if o] or save_times
        save_sec = mx(statistics.mean(ok_times))
        save_max = mx(max(ok_times))
        step_sec = mx(statistics.median(step_times))
        loss_v = float(loss.float().item())
        per_save_cost = mx(1000.0 * (t_loop / a.steps - statistics.median(step_times)) * a.ckpt_interval)

        # ---------------- the opt-in overlapped snapshot copy: the same loop
        # with the HBM copy on a side stream under the next forward
        cp = ckpt.engine._copier
        save_ov, cost_ov = None, None
        if cuda and cp is not None and not cp.overlap:
            ckpt.wait_latest_checkpoint()
            sync_all()
            cp.overlap = True
            ov_saves, ov_steps = [], []
            n_ov = 3 * a.ckpt_interval
            t1 = time.perf_counter()
            for i in range(n_ov):
                ts = time.perf_counter()
                train_step(False)
                sync_step()
                ov_steps.append(time.perf_counter() - ts)
                if i % a.ckpt_interval == 0:
                    ov_saves.append(save()[0])
            t_ov = time.perf_counter() - t1
            ckpt.wait_latest_checkpoint()
            sync_all()
            cp.overlap = False
            save_ov = round(mx(statistics.mean(ov_saves)), 4)
            cost_ov = round(mx(1000.0 * (t_ov / n_ov - statistics.median(ov_steps)) * a.ckpt_interval), 2)

        # ---------------- time to durable: pause + flush until in shm
        ckpt.wait_latest_checkpoint()
        sync_all()
        t0 = time.perf_counter()
        save()
        ckpt.wait_latest_checkpoint()
        durable = mx(time.perf_counter() - t0)
        cp = ckpt.engine._copier
        flush_gbps = None
        if cp is not None and cp.flush_stats:
            nb, dt = cp.flush_stats[-1]
            flush_gbps = round(nb / dt / 1e9, 1)

        # ---------------- in-process load (warm process; verified bit-exact)
        sync_all()
        third = opt.master if opt.master is not None else opt.exp_avg_sq
        ref_sum = flat.data.float().sum().item(), opt.exp_avg.sum().item(), third.sum().item()
        replicas_identical = True
        if world > 1:
            chk = torch.tensor([ref_sum[0], ref_sum[2]], dtype=torch.float64, device=cdev)
            lo_, hi_ = chk.clone(), chk.clone()
            dist.all_reduce(lo_, op=dist.ReduceOp.MIN)
            dist.all_reduce(hi_, op=dist.ReduceOp.MAX)
            replicas_identical = bool(torch.equal(lo_, hi_))
        flat.data.zero_()
        opt.exp_avg.zero_()
        third.zero_()
        sync_all()
        t0 = time.perf_counter()
        ckpt.load_checkpoint(target=state())
        if cuda:
            torch.cuda.synchronize()
        load_warm = mx(time.perf_counter() - t0)
        got = flat.data.float().sum().item(), opt.exp_avg.sum().item(), third.sum().item()
        load_ok = all(abs(x - y) <= 1e-6 * max(1.0, abs(x)) for x, y in zip(ref_sum, got))
        ckpt_bytes = ckpt.engine._shm_handler.payload_size

        emit({"event": "phase0", "world": world, "dtype": "bf16" if cuda else "fp32", "desc": desc,
              "params": nparams, "t_timed": t_timed, "save_sec_mean": save_sec, "save_sec_max": save_max,
              "step_sec": step_sec, "loss": round(loss_v, 4), "durable_sec": durable, "flush_gbps": flush_gbps,
              "load_sec_warm": load_warm, "load_ok": load_ok, "replicas_identical": replicas_identical,
              "ckpt_bytes": ckpt_bytes, "first_save_sec": first_save, "timed_saves": len(save_times),
              "timed_saves_ok": timed_ok, "skipped_saves_timed": skipped_timed, "rehearsal": rehearsal,
              "backend": backend, "slices": ckpt.engine._num_slices, "hbm_plan": getattr(ckpt.engine, "hbm_plan", None),
              "host_plan": getattr(ckpt.engine, "host_plan", None),
              "gather": ckpt.engine._gather_group is not None, "pg": pg_info,
              "optimizer_update": "under next forward" if opt._overlap is not None else "compute stream",
              "snapshot_copy": "overlapped (fenced by the next optimizer step)" if ckpt.engine._copier is not None
              and ckpt.engine._copier.overlap else "in the pause",
              "per_save_cost_ms": round(per_save_cost, 2), "save_sec_overlapped": save_ov,
              "per_save_cost_ms_overlapped": cost_ov})

        # ---------------- DISK persist (agent: torch.save archive written from
        # shm with parallel pwrite) while training continues: persist time and
        # step-time interference (steps measured while it is in flight)
        if not a.no_persist:
            tracker = os.path.join(a.ckpt_dir, CheckpointConstant.TRACER_FILE_NAME)
            sync_all()
            persist_step = step
            persist_t0 = time.time()
            ckpt.save_checkpoint(step, state(), storage_type=StorageType.DISK)
            during, persist_done = [], None
            # a persist that never lands (disk full, storage error) must not
            # hang the run: give up after DWAMD_BENCH_PERSIST_TIMEOUT_S
            persist_deadline = time.time() + float(os.environ.get("DWAMD_BENCH_PERSIST_TIMEOUT_S", "300"))
            while persist_done is None:
                if len(during) < 400:
                    ts = time.perf_counter()
                    train_step(False)
                    sync_step()
                    during.append(time.perf_counter() - ts)
                else:
                    time.sleep(0.01)
                done_here = 0  # rank 0 decides for all: 1 durable, 2 past the deadline
                if rank == 0:
                    try:
                        with open(tracker) as f:
                            done_here = 1 if f.read().strip() == str(persist_step) else 0
                    except OSError:
                        pass
                    if not done_here and time.time() > persist_deadline:
                        done_here = 2
                if world > 1:
                    t = torch.tensor([done_here], device=cdev)
                    dist.broadcast(t, 0)
                    done_here = int(t.item())
                if done_here == 1:
                    persist_done = time.time() - persist_t0
                elif done_here == 2:
                    log(f"[rank {rank}] persist of step {persist_step} not durable after the deadline")
                    break
            med = mx(statistics.median(during)) if during else None
            emit({"event": "persisted", "persist_sec": persist_done, "steps_during": len(during),
                  "step_ms_during": round(1000 * med, 2) if med else None,
                  "interference_pct": round(100 * (med / step_sec - 1), 2) if med else None})

            if persist_done is not None:  # (no durable archive: no storage restore to time)
                # ---------------- storage restore (node replaced: shm gone): the
                # persisted archive straight into the live tensors, page cache
                # dropped first and O_DIRECT reads -- the device's read rate
                from dlrover_wuqiong_amd.flash_checkpoint.storage_loader import drop_file_cache

                path = os.path.join(a.ckpt_dir, str(persist_step), "rank_0.pt")  # DDP: one node copy
                sync_all()
                flat.data.zero_()
                opt.exp_avg.zero_()
                third.zero_()
                try:
                    drop_file_cache(path)
                except OSError:
                    pass
                sync_all()
                t0 = time.perf_counter()
                ckpt.engine._load_from_storage(path, target={CheckpointConstant.MODEL_STATES_NAME: state()})
                if cuda:
                    torch.cuda.synchronize()
                sec = mx(time.perf_counter() - t0)
                from_storage = state_sums()
                storage_src = getattr(ckpt.engine, "last_restore_source", None)
                # the same step from memory (the DISK save snapshotted it to shm
                # first): the two restores must agree bit for bit.  This also puts
                # the live state back to that checkpoint for the fault window.
                ckpt.load_checkpoint(target=state())
                sync_all()
                emit({"event": "storage_load", "sec": sec, "ok": from_storage == state_sums(),
                      "source": storage_src, "stats": getattr(ckpt.engine, "last_storage_load_stats", None)})
        sync_all()
        s0 = step
        emit({"event": "fault_start", "t": time.time(), "s0": s0})
        start_step = step
    else:
        # ---------------- restarted incarnation: restore from the node's memory
        sync_all()
        t0 = time.perf_counter()
        restored = ckpt.load_checkpoint(target=state())
        t_host = time.perf_counter()
        deferred = getattr(ckpt.engine, "last_deferred_restore", None)
        if cuda:
            # with a deferred optimizer-state restore only the compute
            # stream's copies (model) block; the rest lands during step 1
            (torch.cuda.current_stream() if deferred is not None else torch.cuda).synchronize()
        restore_dev = time.perf_counter() - t_host
        restore_block = time.perf_counter() - t0
        step = int(restored.get("step", 0)) if restored else 0
        restore_ok = bool(restored) and step > 0
        if restore_ok:
            di.discard()
        else:
            di.replay()  # nothing restored: the parameters still need their init
        # bit-exact check against the sums incarnation 0 logged right after
        # that save (the last one before the kill)
        want = [e for e in _read_jsonl(step_log) if e["event"] == "saved_sums" and e["rank"] == rank
                and e["step"] == step]
        late_sums = None
        if restore_ok and want:
            if deferred is not None:
                late_sums = state_sums_behind(deferred)  # checked after step 1
            else:
                restore_ok = state_sums() == want[-1]["sums"]
        # load_sec: until every byte is resident (a deferred restore's last
        # copy included; it overlaps step 1, and is collected after it)
        restore_sec = mx(restore_block) if deferred is None else None
        t_restored = time.time()
        emit({"event": "start", "incarnation": incarnation, "t": time.time(), "restored_step": step,
              "restore_sec": restore_sec, "restore_ok": restore_ok if late_sums is None else None,
              "restore_blocking_sec": round(restore_block, 4), "t_proc": t_proc, "t_model": t_model,
              "t_activated": t_act, "t_pg": t_pg, "t_ckpt": t_ckpt, "t_restored": t_restored,
              "build_marks": {k: round(v - t_proc, 3) for k, v in marks.items()},
              "prepin_s": info.get("prepin_s") if info else None, "standby": "deep" if info else "import",
              "pg": pg_info,
              "restore_source": getattr(ckpt.engine, "last_restore_source", None),
              "restore_gather": getattr(ckpt.engine._copier, "last_restore_gather", None),
              "restore_phases": dict(getattr(ckpt.engine, "last_restore_breakdown", {}) or {},
                                     device_wait=round(restore_dev, 4))})
        if not restore_ok:
            log(f"[rank {rank}] restore from memory failed: starting over")
        start_step = step
        s0 = next(e for e in _read_jsonl(step_log) if e["event"] == "fault_start")["s0"]
    if incarnation > 0:
        pending_check = (late_sums, want[-1]["sums"] if want else None, deferred)
    else:
        pending_check = None

    # ---------------- fault window: train + save every interval; rank n-1 dies mid-step
    if incarnation == 0 and a.inject_slow_flush > 0:
        os.environ["DWAMD_FAULT_FLUSH_DELAY_S"] = str(a.inject_slow_flush)
    kill_after = _kill_after(a, s0) if not a.no_fault else -1
    s_end = s0 + a.fault_window
    last_before_kill = kill_after - (kill_after - s0) % a.ckpt_interval if kill_after > 0 else -1
    skipped_w = ckpt.engine.skipped_saves
    saves_after, allocs_after = 0, None
    while step < s_end:
        train_step(True)
        sync_step()
        if pending_check is not None:
            # the deferred restore: residency time and the bit-exact check,
            # both settled behind step 1
            late, wanted, dres = pending_check
            pending_check = None
            res_sec = dres.resident_sec() if dres is not None else None
            ok = (late() == wanted) if late is not None else None
            res_sec = mx(res_sec if res_sec is not None else -1.0)  # collective on every rank
            emit({"event": "restore_late", "rank": rank, "restore_ok": ok,
                  "resident_sec": res_sec if res_sec >= 0 else None})
        save_ms = None
        if (step - s0) % a.ckpt_interval == 0:
            _dt, ok = save()
            save_ms = round(1000 * _dt, 2)
            if not ok:
                emit({"event": "window_skipped", "n": 1, "step": step, "incarnation": incarnation})
            if incarnation > 0:
                saves_after += 1
                if saves_after == 4:
                    allocs_after = dev_allocs() - alloc0
            if incarnation == 0 and step == last_before_kill:
                emit({"event": "saved_sums", "step": step, "rank": rank, "sums": state_sums()}, all_ranks=True)
        emit({"event": "step", "step": step, "t": time.time(), "incarnation": incarnation, "save_ms": save_ms})
    del skipped_w
    # end of the window: every rank's compute done (the background flush of
    # the last checkpoint is not training time and is not waited for)
    if world > 1:
        dist.barrier()
    sync_step()
    cp = ckpt.engine._copier
    # the window's flushes (HBM staging -> shm): queueing delay and duration
    # per flush, for save-wait diagnosis (a save waits when the previous
    # flush of its staging buffer has not landed)
    flushes = []
    for rec in (list(getattr(cp, "flush_log", []) or [])[-12:] if cp is not None else []):
        te, t0, t1, nb = rec[:4]
        f = {"wait_ms": round(1000 * (t0 - te), 1), "ms": round(1000 * (t1 - t0), 1),
             "gbps": round(nb / max(t1 - t0, 1e-9) / 1e9, 1)}
        if len(rec) >= 6:  # queued behind the previous flush / pinned share of the destination
            f["queued_ms"] = round(1000 * (rec[4] - te), 1)
            f["pinned_frac"] = round(rec[5] / max(1, nb), 3)
        flushes.append(f)
    emit({"event": "done", "t": time.time(), "step": step, "start_step": start_step, "incarnation": incarnation,
          "flushes": flushes, "skipped_saves": ckpt.engine.skipped_saves, "gc_pauses": gc_pauses[-20:],
          "device_allocs_after_restart": allocs_after if allocs_after is not None else (
              dev_allocs() - alloc0 if incarnation > 0 else None)})
    sync_all()
    ckpt.close()
    if world > 1:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def main():
    a = parse()
    if os.environ.get(WORKER_ENV) == "1":
        sys.exit(worker(a))
    sys.exit(launcher(a))


if __name__ == "__main__":
    main()
