"""GPT-2 1.5B MLP (8192 x 1600 -> 6400 -> 1600) forward / backward time per
implementation: unfused kernels vs the hipBLASLt epilogue paths."""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return 1000 * (time.perf_counter() - t0) / it


def main():
    from dlrover_wuqiong_amd.ops import mlp as M
    from dlrover_wuqiong_amd.ops.activation import bias_gelu
    from dlrover_wuqiong_amd.ops.linear import linear

    C, T = 1600, 8192
    fc = torch.nn.Linear(C, 4 * C).cuda().bfloat16()
    proj = torch.nn.Linear(4 * C, C).cuda().bfloat16()
    x = torch.randn(T, C, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(T, C, device="cuda", dtype=torch.bfloat16)

    def unfused():
        h = linear(x, fc.weight)
        return proj(bias_gelu(h, fc.bias))

    rows = []
    for name, fn in (("unfused", unfused), ("fused", lambda: M.fused_gelu_mlp(x, fc, proj))):
        for mode in (["-"] if name == "unfused" else ["bgrad", "dgelu", "unfused"]):
            if name == "fused":
                M._BWD_MODE[(T, 4 * C, C)] = mode
            fwd = t(lambda: fn())
            fb = t(lambda: fn().backward(dy))
            rows.append({"impl": name, "bwd_mode": mode, "fwd_ms": round(fwd, 3), "fwd_bwd_ms": round(fb, 3)})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
