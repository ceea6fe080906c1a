"""Rotary position embedding (rotate-half convention) on a host-built
cos/sin table (``csrc/kernels/elementwise.hip:dw_rope``)."""

import torch

from . import _hip

_TABLES = {}


def rope_table(seq_len: int, head_dim: int, base: float = 10000.0, device="cpu"):
    key = (seq_len, head_dim, base, str(device))
    t = _TABLES.get(key)
    if t is None:
        inv = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
        pos = torch.arange(seq_len, dtype=torch.float64)
        freqs = torch.outer(pos, inv)
        t = (freqs.cos().float().to(device).contiguous(), freqs.sin().float().to(device).contiguous())
        _TABLES[key] = t
    return t


def _rope_ref(x, cos, sin, sign=1.0, pos_ids=None):
    # x: [B, S, NH, D]
    D = x.shape[-1]
    h = D // 2
    S = x.shape[1]
    c = cos[:S] if pos_ids is None else cos[pos_ids]
    s = sin[:S] if pos_ids is None else sin[pos_ids]
    if pos_ids is None:
        c = c[None, :, None, :]
        s = s[None, :, None, :]
    else:
        c = c.view(x.shape[0], S, 1, h)
        s = s.view(x.shape[0], S, 1, h)
    s = s * sign
    xf = x.float()
    a, b = xf[..., :h], xf[..., h:]
    return torch.cat([a * c - b * s, b * c + a * s], dim=-1).to(x.dtype)


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, pos_ids):
        x = x.contiguous()
        _hip.require_bf16(x)
        B, S, NH, D = x.shape
        y = torch.empty_like(x)
        pid = pos_ids.to(torch.int32).contiguous() if pos_ids is not None else None
        _hip.check(_hip.lib().dw_rope(_hip.ptr(x), _hip.ptr(y), _hip.ptr(cos), _hip.ptr(sin), B, S, NH, D, 0,
                                      _hip.ptr(pid), cos.shape[0], _hip.stream()), "rope")
        ctx.save_for_backward(cos, sin, pid)
        return y

    @staticmethod
    def backward(ctx, dy):
        cos, sin, pid = ctx.saved_tensors
        dy = dy.contiguous().to(torch.bfloat16)
        B, S, NH, D = dy.shape
        dx = torch.empty_like(dy)
        _hip.check(_hip.lib().dw_rope(_hip.ptr(dy), _hip.ptr(dx), _hip.ptr(cos), _hip.ptr(sin), B, S, NH, D, 1,
                                      _hip.ptr(pid), cos.shape[0], _hip.stream()), "rope_bwd")
        return dx, None, None, None


def _table(t, x, pos_ids):
    # The kernel reads an fp32 [rows, D/2] table.  Callers under FSDP2 mixed
    # precision get the table re-cast to bf16 as a layer input: upcast it here
    # (reading a bf16 table as fp32 walks past its end).
    B, S, NH, D = x.shape
    if t.dim() != 2 or t.shape[1] != D // 2:
        raise _hip.HipKernelError(f"rope table shape {tuple(t.shape)} does not match head_dim {D}")
    if pos_ids is None and t.shape[0] < S:
        raise _hip.HipKernelError(f"rope table has {t.shape[0]} rows < seq_len {S}")
    if pos_ids is not None:
        if pos_ids.numel() != B * S:
            raise _hip.HipKernelError(f"rope pos_ids has {pos_ids.numel()} entries, expected {B * S}")
        if pos_ids.device != x.device or pos_ids.dtype.is_floating_point or pos_ids.dtype == torch.bool:
            raise _hip.HipKernelError(f"rope pos_ids must be an integer tensor on {x.device} "
                                      f"(got {pos_ids.dtype} on {pos_ids.device})")
        # out-of-table positions are clamped by the kernel (never read past the table)
    if t.dtype != torch.float32 or not t.is_contiguous() or t.device != x.device:
        t = t.to(device=x.device, dtype=torch.float32).contiguous()
    return t


def apply_rope(x, cos, sin, pos_ids=None):
    """x: [B, S, NH, D]; cos/sin: [>=S, D/2] (fp32; other dtypes upcast)."""
    if _hip.bf16_path(x):
        x = _hip.bf16(x)
        return _RopeFn.apply(x, _table(cos, x, pos_ids), _table(sin, x, pos_ids), pos_ids)
    return _rope_ref(x, cos, sin, 1.0, pos_ids)


class _QkvRopeFn(torch.autograd.Function):
    """Split of a packed QKV projection + RoPE on q and k in one pass
    (``dw_qkv_rope``); backward: inverse rotation + interleaved write of the
    packed gradient in one pass."""

    @staticmethod
    def forward(ctx, qkv, nh, nkv, cos, sin, pos_ids):
        qkv = qkv.contiguous()
        _hip.require_bf16(qkv)
        B, S, NT, D = qkv.shape
        q = torch.empty(B, S, nh, D, device=qkv.device, dtype=qkv.dtype)
        k = torch.empty(B, S, nkv, D, device=qkv.device, dtype=qkv.dtype)
        v = torch.empty(B, S, nkv, D, device=qkv.device, dtype=qkv.dtype)
        pid = pos_ids.to(torch.int32).contiguous() if pos_ids is not None else None
        _hip.check(_hip.lib().dw_qkv_rope(_hip.ptr(qkv), _hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(cos),
                                          _hip.ptr(sin), B, S, nh, nkv, D, 0, _hip.ptr(pid), cos.shape[0],
                                          _hip.stream()), "qkv_rope")
        ctx.save_for_backward(cos, sin, pid)
        ctx.shape = (B, S, NT, D, nh, nkv)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin, pid = ctx.saved_tensors
        B, S, NT, D, nh, nkv = ctx.shape
        dev = (dq if dq is not None else dk if dk is not None else dv).device

        def g(t, heads):
            if t is None:
                return torch.zeros(B, S, heads, D, device=dev, dtype=torch.bfloat16)
            return t.contiguous().to(torch.bfloat16)

        dq, dk, dv = g(dq, nh), g(dk, nkv), g(dv, nkv)
        dqkv = torch.empty(B, S, NT, D, device=dev, dtype=torch.bfloat16)
        _hip.check(_hip.lib().dw_qkv_rope(_hip.ptr(dqkv), _hip.ptr(dq), _hip.ptr(dk), _hip.ptr(dv), _hip.ptr(cos),
                                          _hip.ptr(sin), B, S, nh, nkv, D, 1, _hip.ptr(pid), cos.shape[0],
                                          _hip.stream()), "qkv_rope_bwd")
        return dqkv, None, None, None, None, None


def qkv_split_rope(qkv, nh: int, nkv: int, cos, sin, pos_ids=None):
    """qkv: [B, S, nh + 2 nkv, D] (a packed QKV projection, heads ordered
    q | k | v) -> contiguous (rope(q), rope(k), v), each [B, S, heads, D]."""
    if _hip.bf16_path(qkv):
        qkv = _hip.bf16(qkv)
        q4 = qkv[:, :, :nh]
        return _QkvRopeFn.apply(qkv, nh, nkv, _table(cos, q4, pos_ids), _table(sin, q4, pos_ids), pos_ids)
    q, k, v = qkv.split([nh, nkv, nkv], dim=2)
    return _rope_ref(q, cos, sin, 1.0, pos_ids), _rope_ref(k, cos, sin, 1.0, pos_ids), v.contiguous()
