"""Flash attention (HIP/MFMA kernels ``attn_fwd.hip`` / ``attn_bwd.hip``).

Layout is BSHD (``[batch, seq, heads, head_dim]``): exactly what a fused QKV
projection produces after a view, so no transposes are materialised.  GQA is
supported (k/v with fewer heads).  head_dim 64 or 128.

Parity: reference ATorch ``FlashAttnModule`` / ``flash_attn_func`` usage
(atorch/atorch/modules/transformer/layers.py; distributed_transformer/
distributed_attention.py for the sequence-parallel variant).
"""

import ctypes
import math

import torch
import torch.nn.functional as F

from . import _hip


def _bs_rs(t: torch.Tensor):
    """(batch stride, sequence-row stride) of a BSHD view whose (head, dim)
    block is dense."""
    B, S, H, D = t.shape
    assert t.stride(3) == 1 and t.stride(2) == D, "head/dim must be dense"
    return t.stride(0), t.stride(1)


def _strides(*ts) -> ctypes.Array:
    vals = []
    for t in ts:
        vals.extend(_bs_rs(t))
    return (ctypes.c_longlong * len(vals))(*vals)


def _dense_hd(t: torch.Tensor) -> torch.Tensor:
    return t if (t.stride(3) == 1 and t.stride(2) == t.shape[3]) else t.contiguous()


class _FlashAttnQKVPackedFn(torch.autograd.Function):
    """q/k/v are views of one [B, S, 3, H, D] tensor: no split copies in the
    forward, and the backward writes dq/dk/dv straight into one packed
    gradient (no concatenation)."""

    @staticmethod
    def forward(ctx, qkv, causal, scale):
        _hip.require_bf16(qkv)
        B, S, _three, H, D = qkv.shape
        if qkv.stride(4) != 1 or qkv.stride(3) != D or qkv.stride(2) != H * D:
            qkv = qkv.contiguous()
        q, k, v = qkv.unbind(2)
        o = torch.empty(B, S, H, D, device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty(B, H, S, device=qkv.device, dtype=torch.float32)
        _hip.check(_hip.lib().dw_attn_fwd_strided(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o),
                                                  _hip.ptr(lse), B, S, H, H, D, _strides(q, k, v, o), int(causal),
                                                  float(scale), 0, _hip.stream()), "attn_fwd")
        ctx.save_for_backward(qkv, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        do = _dense_hd(do.to(torch.bfloat16))
        B, S, _three, H, D = qkv.shape
        q, k, v = qkv.unbind(2)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv.unbind(2)
        L = _hip.lib()
        ws = torch.empty(L.dw_attn_bwd_workspace(B, S, H, D), device=qkv.device, dtype=torch.uint8)
        _hip.check(L.dw_attn_bwd_strided(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(do),
                                         _hip.ptr(lse), _hip.ptr(dq), _hip.ptr(dk), _hip.ptr(dv), _hip.ptr(ws),
                                         B, S, H, H, D, _strides(q, k, v, o, do, dq, dk, dv), int(ctx.causal),
                                         float(ctx.scale), 0, _hip.stream()), "attn_bwd")
        return dqkv, None, None


def flash_attn_qkvpacked_func(qkv, causal: bool = True, softmax_scale=None):
    """qkv: [B, S, 3, H, D] (a fused QKV projection viewed) -> [B, S, H, D]."""
    D = qkv.shape[-1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    if _hip.use_hip(qkv):
        return _FlashAttnQKVPackedFn.apply(qkv, causal, scale)
    q, k, v = qkv.unbind(2)
    return flash_attn_func(q, k, v, causal, scale)


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
