"""Quantize / dequant-reduce HBM bandwidth on one MI355X (qwZ / qgZ kernels).

Prints one JSON line per case: GB/s counts the bytes the kernel must move
(read bf16 + write codes + params; dequant-reduce reads N code chunks and
writes the reduced bf16 shard).
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.ops.quantization import dequant_reduce, quantize  # noqa: E402


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


def main():
    n = 1 << 28  # 256 Mi elements: a 512 MB bf16 gradient bucket
    x = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    for bits in (8, 4):
        gs = 2048
        t = timed(lambda: quantize(x, n // gs, bits))
        moved = 2 * n + n * bits / 8 + (n // gs) * 8
        print(json.dumps({"op": "quantize", "bits": bits, "elems": n, "group": gs, "ms": round(t * 1e3, 3),
                          "gbps": round(moved / t / 1e9, 1)}), flush=True)
        n_src, m = 8, n // 8
        codes, params = quantize(x, n // gs, bits)
        out = torch.empty(m, device="cuda", dtype=torch.bfloat16)
        t = timed(lambda: dequant_reduce(codes, params, n_src, m, gs, bits, out=out))
        moved = n * bits / 8 + (n // gs) * 8 + 2 * m
        print(json.dumps({"op": "dequant_reduce", "bits": bits, "n_src": n_src, "elems_out": m, "ms": round(t * 1e3, 3),
                          "gbps": round(moved / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
