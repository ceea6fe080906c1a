"""Flash attention fwd/bwd timing (TFLOP/s, causal FLOPs halved) for the
GPT2-1.5B shape and Llama-style D=128 GQA shapes."""
import json
import math

import torch

import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.ops.attention import flash_attn_func, flash_attn_qkvpacked_func


def t(fn, it=20, reps=5):
    """Median over ``reps`` runs of ``it`` back-to-back calls (ms per call)."""
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        s.record()
        for _ in range(it):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / it)
    return sorted(out)[reps // 2]


def main():
    for (B, S, H, HKV, D, packed) in [(8, 1024, 25, 25, 64, True), (8, 1024, 25, 25, 64, False),
                                      (4, 4096, 32, 8, 128, False), (1, 8192, 32, 8, 128, False)]:
        dev = "cuda"
        if packed:
            qkv = torch.randn(B, S, 3, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
            f = lambda: flash_attn_qkvpacked_func(qkv, causal=True)  # noqa: E731
            ins = [qkv]
        else:
            q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
            k = torch.randn(B, S, HKV, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
            v = torch.randn(B, S, HKV, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
            f = lambda: flash_attn_func(q, k, v, causal=True)  # noqa: E731
            ins = [q, k, v]
        o = f()
        do = torch.randn_like(o)
        tf = t(f)
        tb = t(lambda: torch.autograd.grad(o, ins, do, retain_graph=True))
        fl = 4 * B * H * S * S * D / 2
        # torch SDPA (ROCm flash backend) on the same problem, [B, H, S, D] layout
        qs = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        ks = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        vs = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        fs = lambda: torch.nn.functional.scaled_dot_product_attention(qs, ks, vs, is_causal=True)  # noqa: E731
        try:
            os_ = fs()
            dos = torch.randn_like(os_)
            sf = t(fs)
            sb = t(lambda: torch.autograd.grad(os_, [qs, ks, vs], dos, retain_graph=True))
        except Exception:
            sf = sb = float("nan")
        print(json.dumps({"B": B, "S": S, "H": H, "HKV": HKV, "D": D, "packed": packed, "fwd_us": round(tf * 1e3, 1),
                          "bwd_us": round(tb * 1e3, 1), "fwd_tflops": round(fl / tf / 1e9, 1),
                          "bwd_tflops": round(2.5 * fl / tb / 1e9, 1),
                          "sdpa_fwd_tflops": round(fl / sf / 1e9, 1), "sdpa_bwd_tflops": round(2.5 * fl / sb / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
