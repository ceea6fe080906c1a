"""Flash attention (HIP/MFMA kernels ``attn_fwd.hip`` / ``attn_bwd.hip``).

Layout is BSHD (``[batch, seq, heads, head_dim]``): exactly what a fused QKV
projection produces after a view, so no transposes are materialised.  GQA is
supported (k/v with fewer heads).  head_dim 64 or 128.

Parity: reference ATorch ``FlashAttnModule`` / ``flash_attn_func`` usage
(atorch/atorch/modules/transformer/layers.py; distributed_transformer/
distributed_attention.py for the sequence-parallel variant).
"""

import math

import torch
import torch.nn.functional as F

from . import _hip


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        _hip.require_bf16(q, k, v)
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, S, H, D = q.shape
        HKV = k.shape[2]
        o = torch.empty_like(q)
        lse = torch.empty(B, H, S, device=q.device, dtype=torch.float32)
        _hip.check(_hip.lib().dw_attn_fwd(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(lse),
                                          B, S, H, HKV, D, int(causal), float(scale), 0, _hip.stream()),
                   "attn_fwd")
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal = causal
        ctx.scale = scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        do = do.contiguous().to(torch.bfloat16)
        B, S, H, D = q.shape
        HKV = k.shape[2]
        L = _hip.lib()
        ws = torch.empty(L.dw_attn_bwd_workspace(B, S, H, D), device=q.device, dtype=torch.uint8)
        dq = torch.empty_like(q)
        dk = torch.empty_like(k)
        dv = torch.empty_like(v)
        _hip.check(L.dw_attn_bwd(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(do), _hip.ptr(lse),
                                 _hip.ptr(dq), _hip.ptr(dk), _hip.ptr(dv), _hip.ptr(ws), None, B, S, H, HKV, D,
                                 int(ctx.causal), float(ctx.scale), 0, _hip.stream()), "attn_bwd")
        return dq, dk, dv, None, None


def attention_reference(q, k, v, causal=True, softmax_scale=None):
    """fp32 math reference (BSHD)."""
    B, S, H, D = q.shape
    HKV = k.shape[2]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    if HKV != H:
        kf = kf.repeat_interleave(H // HKV, dim=1)
        vf = vf.repeat_interleave(H // HKV, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vf)
    return o.transpose(1, 2).to(q.dtype)


def flash_attn_func(q, k, v, causal: bool = True, softmax_scale=None):
    """q: [B, S, H, D]; k, v: [B, S, Hkv, D] -> [B, S, H, D]."""
    D = q.shape[-1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    if _hip.use_hip(q):
        return _FlashAttnFn.apply(q, k, v, causal, scale)
    # CPU execution path
    if k.shape[2] != q.shape[2]:
        return attention_reference(q, k, v, causal, scale)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                       is_causal=causal, scale=scale)
    return o.transpose(1, 2)
