"""Host-side profile of the flash-checkpoint save pause (GPT2-1.5B flat DDP
state, 1 GPU): cProfile of ``DdpCheckpointer.save_checkpoint`` + the
compute-stream sync, after warm-up saves.

    python scripts/prof_save_host.py --model gpt2-1.5b --saves 10
"""

import argparse
import cProfile
import io
import json
import os
import pstats
import statistics
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-1.5b")
    ap.add_argument("--saves", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/prof_save_host.txt")
    ap.add_argument("--no-cprofile", action="store_true", help="plain timings (no profiler overhead)")
    a = ap.parse_args()
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    cfg = GPT2Config.named(a.model)
    with torch.device(dev):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model, dtype=torch.bfloat16, device=dev)
    opt = FusedAdamW(flat, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0)
    flat.grad.normal_()
    opt.step()
    ckpt = DdpCheckpointer(tempfile.mkdtemp(prefix="prof_save_"))
    step = 0

    def state():
        return {"model": model.state_dict(), "optimizer": opt.state_dict(), "step": step}

    def save():
        t0 = time.perf_counter()
        ckpt.save_checkpoint(step, state(), storage_type=StorageType.MEMORY)
        torch.cuda.current_stream().synchronize()
        return time.perf_counter() - t0

    for _ in range(4):
        step += 1
        opt.step()
        save()
        ckpt.wait_latest_checkpoint()
    times, parts = [], []
    pr = cProfile.Profile()
    for _ in range(a.saves):
        step += 1
        opt.step()
        torch.cuda.current_stream().synchronize()
        t0 = time.perf_counter()
        sd = state()
        t1 = time.perf_counter()
        if not a.no_cprofile:
            pr.enable()
        ckpt.save_checkpoint(step, sd, storage_type=StorageType.MEMORY)
        if not a.no_cprofile:
            pr.disable()
        t2 = time.perf_counter()
        torch.cuda.current_stream().synchronize()
        t3 = time.perf_counter()
        times.append(t3 - t0)
        parts.append((t1 - t0, t2 - t1, t3 - t2))
        ckpt.wait_latest_checkpoint()
    s = io.StringIO()
    if not a.no_cprofile:
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
    res = {"save_ms_mean": 1000 * statistics.mean(times), "state_dict_ms": 1000 * statistics.mean(p[0] for p in parts),
           "save_call_ms": 1000 * statistics.mean(p[1] for p in parts),
           "gpu_wait_ms": 1000 * statistics.mean(p[2] for p in parts),
           "speculate": os.environ.get("DWAMD_CKPT_SPECULATE", "1"), "cprofile": not a.no_cprofile}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        f.write(json.dumps(res) + "\n" + s.getvalue())
    print(json.dumps(res))
    ckpt.close() if hasattr(ckpt, "close") else None


if __name__ == "__main__":
    main()
