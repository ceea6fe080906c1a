"""Time every GEMM of a GPT2-1.5B training step in isolation (fwd + both
backward GEMMs of F.linear with bias), bf16, to find slow hipBLASLt picks."""
import json
import sys

import torch
import torch.nn.functional as F


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    M = 8192
    out = []
    for (k, n, bias) in [(1600, 4800, True), (1600, 1600, True), (1600, 6400, True), (6400, 1600, True),
                         (1600, 50304, False)]:
        x = torch.randn(M, k, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        b = torch.randn(n, device="cuda", dtype=torch.bfloat16, requires_grad=True) if bias else None
        dy = torch.randn(M, n, device="cuda", dtype=torch.bfloat16)
        t_f = bench(lambda: F.linear(x, w, b))
        t_dx = bench(lambda: dy @ w)
        t_dw = bench(lambda: dy.t() @ x)
        y = F.linear(x, w, b)
        t_bw = bench(lambda: torch.autograd.grad(y, [x, w] + ([b] if bias else []), dy, retain_graph=True))
        fl = 2 * M * k * n
        out.append({"k": k, "n": n, "fwd_ms": round(t_f, 4), "dx_ms": round(t_dx, 4), "dw_ms": round(t_dw, 4),
                    "autograd_bwd_ms": round(t_bw, 4), "fwd_tflops": round(fl / t_f / 1e9, 1),
                    "dw_tflops": round(fl / t_dw / 1e9, 1), "bwd_tflops": round(2 * fl / t_bw / 1e9, 1)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    sys.exit(main())
