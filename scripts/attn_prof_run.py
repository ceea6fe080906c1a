"""Run attention fwd+bwd for rocprof kernel timing (one shape per argv)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.ops.attention import flash_attn_func, flash_attn_qkvpacked_func  # noqa: E402

fwd_only = "--fwd" in sys.argv
packed = "--packed" in sys.argv  # q/k/v as views of one [B, S, 3, H, D] (HKV = H)
for spec in [a for a in sys.argv[1:] if not a.startswith("--")]:
    B, S, H, HKV, D = map(int, spec.split(","))
    if packed:
        qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        f = lambda: flash_attn_qkvpacked_func(qkv, causal=True)  # noqa: E731
    else:
        q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        f = lambda: flash_attn_func(q, k, v, causal=True)  # noqa: E731
    for _ in range(5):
        if fwd_only:
            with torch.no_grad():
                o = f()
            continue
        o = f()
        o.backward(torch.ones_like(o))
    torch.cuda.synchronize()
print("done")
