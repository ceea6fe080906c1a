"""bf16 nn.Linear vs Fp8Linear (FP8 GEMMs + fused cast/amax) fwd + bwd on
GPT2-1.5B / Llama-8B projection shapes, 1x MI355X."""
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.ops import fp8  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    for (T, K, N) in [(8192, 1600, 6400), (8192, 6400, 1600), (8192, 1600, 4800), (8192, 4096, 14336),
                      (8192, 14336, 4096)]:
        lin = nn.Linear(K, N, device="cuda", dtype=torch.bfloat16)
        f8 = fp8.Fp8Linear(lin)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        g = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)

        def run(m):
            y = m(x)
            y.backward(g)

        tb = timeit(lambda: run(lin))
        t8 = timeit(lambda: (run(f8), fp8.fp8_update()))
        fl = 6 * T * K * N
        print(json.dumps({"T": T, "K": K, "N": N, "bf16_ms": round(tb, 3), "fp8_ms": round(t8, 3),
                          "bf16_tflops": round(fl / tb / 1e9, 1), "fp8_tflops": round(fl / t8 / 1e9, 1),
                          "speedup": round(tb / t8, 2)}), flush=True)


if __name__ == "__main__":
    main()
