#!/usr/bin/env python
"""Where does a cold replacement worker's first training step lose time?

GPT2-1.5B (the bench model: bf16 + fp32 master + AdamW flat state, B=8,
S=1024), each variant in a FRESH child process that first does what the
import-mode standby does before activation (import torch + this package,
HIP init, one small GEMM, load the kernel library) plus the variant's extra
warm-up, then builds the model and times its first three steps:

  record      -- also records the warm profile (GEMMs of step 2 + peak
                 allocator footprint) to --profile
  standby     -- the plain import standby
  nodefer     -- + HIP_ENABLE_DEFERRED_LOADING=0 (every code object loaded
                 at start-up; not in the default list: the eager load
                 segfaults in the HIP runtime on this image, rc -11)
  preload     -- + this package's kernel code objects force-loaded
  reserve     -- + the recorded footprint held in the caching allocator
  replay      -- + the recorded GEMMs replayed
  full        -- replay + preload + reserve (what the standby now does)

The parent never touches the GPU.  Prints one JSON line per variant.
"""

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def child(a):
    t0 = time.time()
    import torch

    from dlrover_wuqiong_amd.elastic_agent import standby, warm_profile

    standby._preload()
    assert standby._gpu_init("0")
    extra = {}
    v = a.variant
    prof = None
    if v in ("replay", "full", "reserve"):
        with open(a.profile) as f:
            prof = json.load(f)
    if v in ("preload", "full"):
        extra["preload_s"] = round(warm_profile.preload_kernel_library(), 3)
    if v in ("replay", "full"):
        extra["replay"] = warm_profile.replay(prof)
    if v in ("reserve", "full"):
        t = time.perf_counter()
        n = warm_profile.reserve_bytes(prof, 0)
        x = torch.empty(n, dtype=torch.uint8, device="cuda")
        del x
        torch.cuda.synchronize()
        extra["reserve_s"] = round(time.perf_counter() - t, 3)
        extra["reserve_gb"] = round(n / 2**30, 1)
    t_ready = time.time()
    # ---- activation: what the training script does from the top
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.ddp import FlatDDP
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    torch.cuda.set_stream(torch.cuda.Stream())
    t_a = time.perf_counter()
    torch.manual_seed(1234)
    cfg = GPT2Config.named("gpt2-1.5b")
    with torch.device("cuda"):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model, dtype=torch.bfloat16, device=torch.device("cuda"))
    opt = FusedAdamW(flat, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0)
    ddp = FlatDDP(model, flat, bucket_mb=128)
    data = torch.randint(0, cfg.vocab_size, (a.batch, 1025), device="cuda")
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t_a
    steps = []
    for i in range(3):
        if i == 1 and v == "record":
            from torch.optim.optimizer import register_optimizer_step_post_hook

            rec = warm_profile._make_recorder()
            rec.__enter__()
            done = {}

            def stop(*_x, **_k):
                if "r" not in done:
                    rec.__exit__(None, None, None)
                    done["r"] = 1

            h = register_optimizer_step_post_hook(stop)
        t = time.perf_counter()
        loss = ddp(data[:, :-1], data[:, 1:])
        loss.backward()
        ddp.finish_gradient_sync()
        opt.step()
        flat.zero_grad()
        torch.cuda.current_stream().synchronize()
        steps.append(round(time.perf_counter() - t, 4))
        if i == 1 and v == "record":
            h.remove()
            prof = {"version": 1, "gemms": list(rec.seen.values()), "gemm_calls": rec.calls,
                    "max_reserved": int(torch.cuda.max_memory_reserved()),
                    "max_allocated": int(torch.cuda.max_memory_allocated())}
            with open(a.profile, "w") as f:
                json.dump(prof, f)
            extra["gemms"] = len(prof["gemms"])
            extra["gemm_calls"] = prof["gemm_calls"]
            extra["max_reserved_gb"] = round(prof["max_reserved"] / 2**30, 1)
    print(json.dumps({"variant": v, "standby_init_s": round(t_ready - t0, 2), "build_s": round(build_s, 3),
                      "step_s": steps, "first_step_excess_s": round(steps[0] - steps[2], 3), **extra}), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", default="")
    p.add_argument("--variants", default="record,standby,preload,reserve,replay,full")
    p.add_argument("--profile", default="/tmp/dwamd_warm_profile.json")
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--out", default="")
    a = p.parse_args()
    if a.variant:
        return child(a)
    lines = []
    for v in a.variants.split(","):
        env = dict(os.environ)
        if v == "nodefer":
            env["HIP_ENABLE_DEFERRED_LOADING"] = "0"
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--variant", v, "--profile", a.profile,
                            "--batch", str(a.batch)], env=env, stdout=subprocess.PIPE, text=True, timeout=300)
        out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        line = out[-1] if out else json.dumps({"variant": v, "rc": r.returncode})
        print(line, flush=True)
        lines.append(line)
        if r.returncode != 0:
            return r.returncode
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
