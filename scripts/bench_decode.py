"""Decode benchmarks (1 GPU): split-KV decode attention bandwidth, and the
RL hybrid engine's generation throughput (graph replay vs eager vs full
forward per token) on a random-init Llama.

    python scripts/bench_decode.py --model llama3-8b --batch 8 --prompt 128 --new 128
"""

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--new", type=int, default=128)
    ap.add_argument("--out", default="gpurun_out/bench_decode.jsonl")
    a = ap.parse_args()
    from dlrover_wuqiong_amd.atorch.rl.hybrid_engine import HybridEngine
    from dlrover_wuqiong_amd.atorch.rl.trainer import sample
    from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig
    from dlrover_wuqiong_amd.ops.attention import decode_attention

    rows = []
    # ---- kernel: bytes of K+V read per call / time
    for B, H, HKV, D, L in ((8, 32, 8, 128, 4096), (8, 32, 8, 128, 16384), (32, 64, 8, 128, 2048),
                            (8, 25, 25, 64, 1024)):
        q = torch.randn(B, H, D, device="cuda", dtype=torch.bfloat16)
        kc = torch.randn(B, L, HKV, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        lens = torch.full((B,), L, device="cuda", dtype=torch.int32)
        t = timeit(lambda: decode_attention(q, kc, vc, lens))
        tsd = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(
            q.view(B, HKV, H // HKV, 1, D).flatten(1, 2), kc.transpose(1, 2).repeat_interleave(H // HKV, 1),
            vc.transpose(1, 2).repeat_interleave(H // HKV, 1)), iters=5)
        gb = 2 * kc.numel() * 2 / 1e9
        rows.append({"kernel": "decode_attention", "B": B, "H": H, "HKV": HKV, "D": D, "L": L, "us": round(1e6 * t, 1),
                     "GBps": round(gb / t, 1), "sdpa_repeat_kv_us": round(1e6 * tsd, 1)})
        print(json.dumps(rows[-1]), flush=True)
        del kc, vc
    # ---- engine
    torch.manual_seed(0)
    cfg = LlamaConfig.named(a.model)
    with torch.device("cuda"):
        m = Llama(cfg)
    m = m.to(torch.bfloat16).eval()
    p = torch.randint(0, cfg.vocab_size, (a.batch, a.prompt), device="cuda")
    for graph in (True, False):
        eng = HybridEngine(m, a.batch, a.prompt + a.new, use_graph=graph)
        eng.generate(p, 8, temperature=0)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.generate(p, a.new, temperature=0)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rows.append({"engine": "hybrid", "graph": graph, "model": a.model, "batch": a.batch, "prompt": a.prompt,
                     "new": a.new, "sec": round(dt, 3), "tokens_per_s": round(a.batch * a.new / dt, 1),
                     "ms_per_token_step": round(1000 * dt / a.new, 2)})
        print(json.dumps(rows[-1]), flush=True)
        del eng
        torch.cuda.empty_cache()
    n = min(32, a.new)
    with torch.no_grad():
        sample(m, p, 2, temperature=0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sample(m, p, n, temperature=0)
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rows.append({"engine": "full_forward_per_token", "model": a.model, "batch": a.batch, "prompt": a.prompt, "new": n,
                 "sec": round(dt, 3), "tokens_per_s": round(a.batch * n / dt, 1),
                 "ms_per_token_step": round(1000 * dt / n, 2)})
    print(json.dumps(rows[-1]), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
