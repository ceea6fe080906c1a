"""Per-shape GEMM solution selection for the flagship training step.

The plain library GEMMs of the GPT2 / Llama steps (linear forward, dgrad,
wgrad) go to hipBLASLt through PyTorch; its default heuristic picks one
solution per shape from a generic table.  PyTorch's TunableOp times every
hipBLASLt and rocBLAS solution for each (transpose, M, N, K) the step issues
and records the fastest in a CSV; ``dlrover_wuqiong_amd.ops.gemm_tuning``
loads that file read-only (no tuning at run time) in ``bench.py`` and the
trainers.

  python scripts/tune_gemms.py --model gpt2-1.5b            # tune -> configs/tunableop/<model>_gfx950.csv
  python scripts/tune_gemms.py --model gpt2-1.5b --ab 20    # time K steps without / with the table

Tuning runs with a rotating input buffer so the timed solutions see cold
caches, as inside the real step.
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(model_name, B, S):
    import torch

    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if model_name.startswith("llama"):
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig

        cfg = LlamaConfig.named(model_name)
        with torch.device(dev):
            model = Llama(cfg)
        vocab = cfg.vocab_size
    else:
        from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

        cfg = GPT2Config.named(model_name)
        cfg.n_positions = max(cfg.n_positions, S)
        with torch.device(dev):
            model = GPT2(cfg)
        vocab = cfg.vocab_size
    model.to(torch.bfloat16)
    flat = FlatParams(model, dtype=torch.bfloat16, device=dev)
    opt = FusedAdamW(flat, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0)
    data = torch.randint(0, vocab, (B, S + 1), device=dev)

    def step():
        loss = model(data[:, :-1], data[:, 1:])
        loss.backward()
        opt.step()
        flat.zero_grad()
        return loss

    return step


def timed(step, n):
    import torch

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="gpt2-1.5b")
    p.add_argument("--micro-batch", type=int, default=8)
    p.add_argument("--seq", type=int, default=1024)
    p.add_argument("--out", default="")
    p.add_argument("--ab", type=int, default=0, help="A/B: time this many steps without and with the table")
    p.add_argument("--mode", default="", help=argparse.SUPPRESS)  # internal: off | on
    a = p.parse_args()
    from dlrover_wuqiong_amd.ops import gemm_tuning

    out = a.out or gemm_tuning.table_path(a.model)
    import torch
    import torch.cuda.tunable as tun

    if a.mode:
        if a.mode == "on":
            assert gemm_tuning.enable(a.model, path=out), f"no tuning table {out}"
        step = build(a.model, a.micro_batch, a.seq)
        ms = 1000 * timed(step, a.ab)
        print(json.dumps({"model": a.model, "tuned": a.mode == "on", "step_ms": round(ms, 2),
                          "n_tuned": len(tun.get_results()) if a.mode == "on" else 0}), flush=True)
        return
    if a.ab:
        import subprocess

        for mode in ("off", "on"):
            rc = subprocess.call([sys.executable, __file__, "--model", a.model, "--micro-batch", str(a.micro_batch),
                                  "--seq", str(a.seq), "--out", out, "--ab", str(a.ab), "--mode", mode])
            if rc != 0:
                sys.exit(rc)
        return
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(out, False)
    tun.set_max_tuning_duration(40)     # ms per solution
    tun.set_max_tuning_iterations(50)
    tun.set_rotating_buffer_size(512)   # MB: cold-cache timings
    step = build(a.model, a.micro_batch, a.seq)
    t0 = time.time()
    step()
    torch.cuda.synchronize()
    print(f"tuned {len(tun.get_results())} GEMM shapes in {time.time() - t0:.1f}s -> {out}", flush=True)
    tun.tuning_enable(False)
    tun.write_file() if hasattr(tun, "write_file") else None


if __name__ == "__main__":
    main()
