"""Numerics of the forward kernel variants (dw_attn_fwd ``flags``) against an
fp32 SDPA reference of the same inputs, incl. ragged lengths, GQA, D 64/128.
    python scripts/attn_pipe_check.py [variant ...]   (default: 0 2)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.ops import _hip  # noqa: E402


def main():
    variants = [int(x) for x in sys.argv[1:]] or [0, 2]
    L = _hip.lib()
    torch.manual_seed(0)
    shapes = [(2, 333, 4, 4, 64, 1), (2, 1024, 4, 4, 64, 1), (1, 300, 2, 2, 64, 0), (2, 77, 3, 3, 64, 1),
              (1, 64, 2, 2, 64, 1), (1, 1, 1, 1, 64, 1), (1, 700, 8, 2, 128, 1), (2, 257, 4, 4, 128, 0),
              (1, 2048, 4, 1, 128, 1)]
    for (B, S, H, HKV, D, causal) in shapes:
        q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
        k = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16)
        qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
        kf = kf.repeat_interleave(H // HKV, 1)
        vf = vf.repeat_interleave(H // HKV, 1)
        ref = torch.nn.functional.scaled_dot_product_attention(qf, kf, vf, is_causal=bool(causal)).transpose(1, 2)
        s = qf @ kf.transpose(-1, -2) * D ** -0.5
        if causal:
            s = s.masked_fill(torch.ones(S, S, device="cuda", dtype=torch.bool).triu(1), float("-inf"))
        lse_ref = torch.logsumexp(s, -1)
        for var in variants:
            o = torch.empty_like(q)
            lse = torch.empty(B, H, S, device="cuda")
            _hip.check(L.dw_attn_fwd(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(lse), B, S, H, HKV,
                                     D, causal, float(D ** -0.5), var, _hip.stream()), "attn_fwd")
            e = (o.float() - ref).abs().max().item()
            el = (lse - lse_ref).abs().max().item()
            print(f"B{B} S{S} H{H}/{HKV} D{D} causal={causal} variant {var}: max|o-ref| {e:.4f} max|lse-ref| {el:.5f}",
                  flush=True)
            assert e < 0.05 and el < 2e-2, (var, e, el)
    print("variants ok")


if __name__ == "__main__":
    main()
