"""Flash attention (HIP/MFMA kernels ``attn_fwd.hip`` / ``attn_bwd.hip``).

Layout is BSHD (``[batch, seq, heads, head_dim]``): exactly what a fused QKV
projection produces after a view, so no transposes are materialised.  GQA is
supported (k/v with fewer heads).  head_dim 64 or 128.

Beyond causal / full masks the same MFMA kernels (an ``EXT`` template
instance, so the plain path is untouched) take sliding windows
(``window_size``), GLM prefix masks (``glm_mask``), an additive bias / mask
(``attn_bias``, broadcastable to [B, H, Sq, Sk]), ALiBi slopes and dropout
(a stateless counter hash of (seed, head, query, key), regenerated in the
backward) -- forward and backward.

Parity: reference ATorch ``FlashAttnModule`` / ``flash_attn_func`` usage
(atorch/atorch/modules/transformer/layers.py:1167-1350: ``flash_attn_with_mask_bias``,
``fa2_with_glm_mask``, ``FlashAttnModule``; distributed_transformer/
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
    if _hip.bf16_path(qkv):
        return _FlashAttnQKVPackedFn.apply(_hip.bf16(qkv), causal, scale)
    q, k, v = qkv.unbind(2)
    return flash_attn_func(q, k, v, softmax_scale=scale, causal=causal)


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


class _AttnExtArgs(ctypes.Structure):
    """ABI of ``AttnExtArgs`` (csrc/kernels/attn_common.h)."""

    _fields_ = [("bias_bs", ctypes.c_longlong), ("bias_hs", ctypes.c_longlong), ("bias_qs", ctypes.c_longlong),
                ("bias", ctypes.c_void_p), ("prefix", ctypes.c_void_p), ("seed", ctypes.c_ulonglong),
                ("offset", ctypes.c_ulonglong), ("win_l", ctypes.c_int), ("win_r", ctypes.c_int),
                ("p_drop", ctypes.c_float), ("pad_", ctypes.c_int), ("alibi", ctypes.c_void_p),
                ("alibi_bs", ctypes.c_longlong)]


def _new_seed() -> int:
    # from torch's CPU generator: torch.manual_seed makes dropout reproducible
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


def _ext_args(bias, prefix, alibi, window, p_drop, seed) -> _AttnExtArgs:
    a = _AttnExtArgs()
    a.win_l, a.win_r = int(window[0]), int(window[1])
    a.p_drop = float(p_drop)
    a.seed = int(seed) & ((1 << 64) - 1)
    a.offset = 0
    if bias is not None:
        a.bias = bias.data_ptr()
        a.bias_bs, a.bias_hs, a.bias_qs = bias.stride(0), bias.stride(1), bias.stride(2)
    if prefix is not None:
        a.prefix = prefix.data_ptr()
    if alibi is not None:
        a.alibi = alibi.data_ptr()
        a.alibi_bs = alibi.stride(0) if alibi.dim() == 2 else 0
    return a


def _prep_bias(bias, B, H, Sq, Sk, device):
    """Additive bias / mask broadcastable to [B, H, Sq, Sk] -> fp32 view with
    stride-0 broadcast dims and a dense key dim (no materialised expand)."""
    if bias is None:
        return None
    if bias.dtype == torch.bool:  # True = keep (SDPA convention)
        bias = torch.zeros(bias.shape, dtype=torch.float32, device=bias.device).masked_fill_(~bias, float("-inf"))
    b = bias.to(device=device, dtype=torch.float32)
    while b.dim() < 4:
        b = b.unsqueeze(0)
    if b.shape[-1] != Sk:
        b = b.expand(*b.shape[:-1], Sk)
    if b.stride(-1) != 1:
        b = b.contiguous()
    return b.expand(B, H, Sq, Sk)


def _prep_alibi(alibi, B, H, device):
    if alibi is None:
        return None
    a = alibi.to(device=device, dtype=torch.float32).contiguous()
    if a.shape not in ((H,), (B, H)):
        raise ValueError(f"alibi_slopes must be [H] or [B, H], got {tuple(a.shape)}")
    return a


class _FlashAttnExtFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, window, bias, prefix, alibi, p_drop, seed):
        _hip.require_bf16(q, k, v)
        q, k, v = _dense_hd(q), _dense_hd(k), _dense_hd(v)
        B, S, H, D = q.shape
        HKV = k.shape[2]
        o = torch.empty(B, S, H, D, device=q.device, dtype=q.dtype)
        lse = torch.empty(B, H, S, device=q.device, dtype=torch.float32)
        args = _ext_args(bias, prefix, alibi, window, p_drop, seed)
        _hip.check(_hip.lib().dw_attn_fwd_ext(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(lse),
                                              B, S, H, HKV, D, _strides(q, k, v, o), int(causal), float(scale),
                                              ctypes.byref(args), _hip.stream()), "attn_fwd_ext")
        ctx.save_for_backward(q, k, v, o, lse, bias, prefix, alibi)
        ctx.meta = (causal, scale, tuple(window), p_drop, seed)
        ctx.mark_non_differentiable(lse)
        return o, lse

    @staticmethod
    def backward(ctx, do, _dlse):
        q, k, v, o, lse, bias, prefix, alibi = ctx.saved_tensors
        causal, scale, window, p_drop, seed = ctx.meta
        do = _dense_hd(do.to(torch.bfloat16))
        B, S, H, D = q.shape
        HKV = k.shape[2]
        L = _hip.lib()
        ws = torch.empty(L.dw_attn_bwd_workspace(B, S, H, D), device=q.device, dtype=torch.uint8)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        args = _ext_args(bias, prefix, alibi, window, p_drop, seed)
        _hip.check(L.dw_attn_bwd_ext(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(do), _hip.ptr(lse),
                                     _hip.ptr(dq), _hip.ptr(dk), _hip.ptr(dv), _hip.ptr(ws), B, S, H, HKV, D,
                                     _strides(q, k, v, o, do, dq, dk, dv), int(causal), float(scale),
                                     ctypes.byref(args), _hip.stream()), "attn_bwd_ext")
        return dq, dk, dv, None, None, None, None, None, None, None, None


def dropout_keep_mask(B: int, H: int, S: int, p: float, seed: int, device="cuda") -> torch.Tensor:
    """The keep mask [B, H, S, S] (bool) the kernels apply for dropout ``p``
    with ``seed`` (dense layout) -- for references and tests."""
    out = torch.empty(B, H, S, S, dtype=torch.uint8, device=device)
    _hip.check(_hip.lib().dw_attn_dropout_mask(_hip.ptr(out), B, H, S, ctypes.c_float(p),
                                               ctypes.c_uint64(int(seed) & ((1 << 64) - 1)), ctypes.c_uint64(0),
                                               _hip.stream()), "attn_dropout_mask")
    return out.bool()


def attention_reference_ext(q, k, v, causal=False, softmax_scale=None, window_size=(-1, -1), attn_bias=None,
                            glm_mask=None, alibi_slopes=None, dropout_p=0.0, keep_mask=None):
    """fp32 math reference of every mask the kernels take (BSHD); rows that
    see no key return 0.  ``keep_mask`` [B, H, S, S] applies dropout."""
    B, S, H, D = q.shape
    HKV = k.shape[2]
    Sk = k.shape[1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    if HKV != H:
        kf = kf.repeat_interleave(H // HKV, dim=1)
        vf = vf.repeat_interleave(H // HKV, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    co = Sk - S
    qi = torch.arange(S, device=q.device)[:, None]
    kj = torch.arange(Sk, device=q.device)[None, :]
    d = kj - (qi + co)
    vis = torch.ones(S, Sk, dtype=torch.bool, device=q.device)
    if causal:
        vis &= d <= 0
    wl, wr = window_size
    if wr >= 0:
        vis &= d <= wr
    if wl >= 0:
        vis &= d >= -wl
    vis = vis[None, None].expand(B, 1, S, Sk)
    if glm_mask is not None:
        vis = vis | (kj[None, None] < glm_mask.to(q.device).view(B, 1, 1, 1))
    if attn_bias is not None:
        s = s + attn_bias.float()
    if alibi_slopes is not None:
        sl = alibi_slopes.float().to(q.device)
        sl = sl.view(1, H, 1, 1) if sl.dim() == 1 else sl.view(B, H, 1, 1)
        s = s - sl * d.abs().float()[None, None]
    s = s.masked_fill(~vis, float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)
    if dropout_p > 0.0 and keep_mask is not None:
        p = p * keep_mask.float() / (1.0 - dropout_p)
    o = torch.matmul(p, vf)
    return o.transpose(1, 2).to(q.dtype)


def flash_attn_func(q, k, v, dropout_p=0.0, softmax_scale=None, causal=False, window_size=(-1, -1),
                    alibi_slopes=None, deterministic=False, return_attn_probs=False, *, glm_mask=None,
                    attn_bias=None, dropout_seed=None):
    """flash-attn's ``flash_attn_func``: q [B, S, H, D]; k, v [B, S, Hkv, D]
    -> [B, S, H, D] (``return_attn_probs``: (out, softmax_lse, None)).
    Extensions: ``glm_mask`` int32 [B] (GLM prefix break points, causal
    only), ``attn_bias`` additive fp32 / bool mask broadcastable to
    [B, H, Sq, Sk] (no gradient).  The kernels are deterministic whatever
    ``deterministic`` says."""
    D = q.shape[-1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    window = tuple(int(w) for w in window_size)
    ext = (dropout_p > 0.0 or window != (-1, -1) or alibi_slopes is not None or glm_mask is not None
           or attn_bias is not None or return_attn_probs)
    if glm_mask is not None and not causal:
        raise ValueError("glm_mask requires causal=True")
    if _hip.bf16_path(q):
        q, k, v = _hip.bf16(q, k, v)
        if not ext:
            return _FlashAttnFn.apply(q, k, v, causal, scale)
        if q.shape[1] != k.shape[1]:
            raise _hip.HipKernelError("extended attention masks need Sq == Sk")
        B, S, H, _ = q.shape
        bias = _prep_bias(attn_bias, B, H, S, S, q.device)
        prefix = glm_mask.to(device=q.device, dtype=torch.int32).contiguous() if glm_mask is not None else None
        alibi = _prep_alibi(alibi_slopes, B, H, q.device)
        seed = (dropout_seed if dropout_seed is not None else _new_seed()) if dropout_p > 0.0 else 0
        o, lse = _FlashAttnExtFn.apply(q, k, v, causal, scale, window, bias, prefix, alibi, float(dropout_p), seed)
        return (o, lse, None) if return_attn_probs else o
    # CPU execution path (same math; dropout from torch's RNG)
    if not ext and k.shape[2] == q.shape[2]:
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                           is_causal=causal, scale=scale)
        return o.transpose(1, 2)
    keep = None
    if dropout_p > 0.0:
        keep = torch.rand(q.shape[0], q.shape[2], q.shape[1], k.shape[1], device=q.device) >= dropout_p
    bias = None
    if attn_bias is not None:
        bias = _prep_bias(attn_bias, q.shape[0], q.shape[2], q.shape[1], k.shape[1], q.device)
    o = attention_reference_ext(q, k, v, causal, scale, window, bias, glm_mask, alibi_slopes, dropout_p, keep)
    return (o, None, None) if return_attn_probs else o


def flash_attn_with_mask_bias(q, k, v, mask=None, bias=None, dropout_p=0.0, softmax_scale=None, causal=False):
    """ATorch ``flash_attn_with_mask_bias`` (layers.py:1167): additive
    ``mask`` [B, H|1, Sq|1, Sk] and ``bias`` [1, H, Sq, Sk] on the MFMA
    kernels (the reference needs a patched FlashAttention-1 for this)."""
    add = None
    if mask is not None and bias is not None:
        add = mask.float() + bias.float()
    elif mask is not None or bias is not None:
        add = mask if mask is not None else bias
    return flash_attn_func(q, k, v, dropout_p=dropout_p, softmax_scale=softmax_scale, causal=causal, attn_bias=add)


def fa2_with_glm_mask(q, k, v, glm_mask=None, dropout_p=0.0, softmax_scale=None, causal=True):
    """ATorch ``fa2_with_glm_mask`` (layers.py:1255): ``glm_mask`` int32 [B]
    break points -- keys before it are visible to every query."""
    if glm_mask is not None and not causal:
        raise ValueError("causal must be True for glm_mask")
    return flash_attn_func(q, k, v, dropout_p=dropout_p, softmax_scale=softmax_scale, causal=causal,
                           glm_mask=glm_mask)


class FlashAttnModule(torch.nn.Module):
    """ATorch ``FlashAttnModule`` (layers.py:1280): dropout active only in
    training; key padding (varlen kernels), GLM break-point masks and
    additive masks / biases."""

    def __init__(self, causal=False, softmax_scale=None, attention_dropout=0.0):
        super().__init__()
        self.causal = causal
        self.softmax_scale = softmax_scale
        self.attention_dropout = attention_dropout

    def forward(self, q, k, v, key_padding_mask=None, glm_mask=None, additive_mask=None, additive_bias=None):
        p = self.attention_dropout if self.training else 0.0
        s_q, s_k = q.shape[1], k.shape[1]
        causal = self.causal and s_q != 1  # single-query decoding
        if s_q != 1 and self.causal and s_q != s_k:
            raise ValueError(f"causal attention needs Sq == Sk (got {s_q}, {s_k}) unless Sq == 1")
        if glm_mask is not None:
            return fa2_with_glm_mask(q, k, v, glm_mask, p, self.softmax_scale, causal=True)
        if additive_mask is not None or additive_bias is not None:
            return flash_attn_with_mask_bias(q, k, v, additive_mask, additive_bias, p, self.softmax_scale, causal)
        if key_padding_mask is None or bool(key_padding_mask.bool().all()):
            return flash_attn_func(q, k, v, dropout_p=p, softmax_scale=self.softmax_scale, causal=causal)
        B = q.shape[0]
        qmask = key_padding_mask[:, -1:] if s_q == 1 else key_padding_mask
        qu, idx, cu_q, mq = unpad_input(q, qmask)
        ku, kidx, cu_k, mk = unpad_input(k, key_padding_mask)
        vu = v.reshape(B * s_k, *v.shape[2:]).index_select(0, kidx)
        o = flash_attn_varlen_func(qu, ku, vu, cu_q, cu_k, mq, mk, dropout_p=p, softmax_scale=self.softmax_scale,
                                   causal=causal)
        return pad_input(o, idx, B, s_q)


# ---------------------------------------------------------------------------
# Variable-length (packed) batches: flash-attn's varlen API on the same
# kernels (``dw_attn_fwd_varlen`` / ``dw_attn_bwd_varlen``; per-block
# sequence extents from cu_seqlens on the device, no padding compute).
def _rows_dense(t: torch.Tensor) -> torch.Tensor:
    """[total, H, D] with dense (H, D): any row stride is fine."""
    return t if (t.stride(2) == 1 and t.stride(1) == t.shape[2]) else t.contiguous()


def _row_strides(*ts) -> ctypes.Array:
    return (ctypes.c_longlong * len(ts))(*[t.stride(0) for t in ts])


class _FlashAttnVarlenFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, cu_q, cu_k, max_sq, max_sk, causal, scale):
        _hip.require_bf16(q, k, v)
        q, k, v = _rows_dense(q), _rows_dense(k), _rows_dense(v)
        cu_q = cu_q.to(device=q.device, dtype=torch.int32).contiguous()
        cu_k = cu_k.to(device=q.device, dtype=torch.int32).contiguous()
        total_q, H, D = q.shape
        HKV = k.shape[1]
        B = cu_q.numel() - 1
        o = torch.empty(total_q, H, D, device=q.device, dtype=q.dtype)
        lse = torch.empty(H, total_q, device=q.device, dtype=torch.float32)
        _hip.check(_hip.lib().dw_attn_fwd_varlen(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(lse),
                                                 _hip.ptr(cu_q), _hip.ptr(cu_k), B, int(max_sq), total_q, H, HKV, D,
                                                 _row_strides(q, k, v, o), int(causal), float(scale), _hip.stream()),
                   "attn_fwd_varlen")
        ctx.save_for_backward(q, k, v, o, lse, cu_q, cu_k)
        ctx.meta = (int(max_sq), int(max_sk), bool(causal), float(scale))
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, cu_q, cu_k = ctx.saved_tensors
        max_sq, max_sk, causal, scale = ctx.meta
        do = _rows_dense(do.to(torch.bfloat16))
        total_q, H, D = q.shape
        total_k, HKV = k.shape[0], k.shape[1]
        B = cu_q.numel() - 1
        L = _hip.lib()
        ws = torch.empty(L.dw_attn_bwd_workspace(B, max(max_sq, max_sk), H, D), device=q.device, dtype=torch.uint8)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _hip.check(L.dw_attn_bwd_varlen(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(do),
                                        _hip.ptr(lse), _hip.ptr(dq), _hip.ptr(dk), _hip.ptr(dv), _hip.ptr(ws),
                                        _hip.ptr(cu_q), _hip.ptr(cu_k), B, max_sq, max_sk, total_q, total_k, H, HKV,
                                        D, _row_strides(q, k, v, o, do, dq, dk, dv), int(causal), float(scale),
                                        _hip.stream()), "attn_bwd_varlen")
        return dq, dk, dv, None, None, None, None, None, None


def varlen_attention_reference(q, k, v, cu_seqlens_q, cu_seqlens_k, causal=False, softmax_scale=None):
    """fp32 reference of the packed layout (bottom-right causal alignment)."""
    H, D = q.shape[1], q.shape[2]
    HKV = k.shape[1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    cq, ck = cu_seqlens_q.tolist(), cu_seqlens_k.tolist()
    out = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
    for b in range(len(cq) - 1):
        qs, ks = q[cq[b]:cq[b + 1]].float(), k[ck[b]:ck[b + 1]].float()
        vs = v[ck[b]:ck[b + 1]].float()
        sq, sk = qs.shape[0], ks.shape[0]
        if sq == 0:
            continue
        if HKV != H:
            ks = ks.repeat_interleave(H // HKV, dim=1)
            vs = vs.repeat_interleave(H // HKV, dim=1)
        s = torch.einsum("qhd,khd->hqk", qs, ks) * scale
        if causal:
            qi = torch.arange(sq, device=q.device)[:, None]
            kj = torch.arange(sk, device=q.device)[None, :]
            s = s.masked_fill(kj > qi + (sk - sq), float("-inf"))
        p = torch.softmax(s, dim=-1).nan_to_num(0.0)  # rows with no visible key -> 0
        out[cq[b]:cq[b + 1]] = torch.einsum("hqk,khd->qhd", p, vs)
    return out.to(q.dtype)


class _FlashAttnVarlenExtFn(torch.autograd.Function):
    """Packed batches with sliding window / ALiBi / dropout (hash index space:
    packed query and key rows)."""

    @staticmethod
    def forward(ctx, q, k, v, cu_q, cu_k, max_sq, max_sk, causal, scale, window, alibi, p_drop, seed):
        _hip.require_bf16(q, k, v)
        q, k, v = _rows_dense(q), _rows_dense(k), _rows_dense(v)
        cu_q = cu_q.to(device=q.device, dtype=torch.int32).contiguous()
        cu_k = cu_k.to(device=q.device, dtype=torch.int32).contiguous()
        total_q, H, D = q.shape
        total_k, HKV = k.shape[0], k.shape[1]
        B = cu_q.numel() - 1
        o = torch.empty(total_q, H, D, device=q.device, dtype=q.dtype)
        lse = torch.empty(H, total_q, device=q.device, dtype=torch.float32)
        args = _ext_args(None, None, alibi, window, p_drop, seed)
        _hip.check(_hip.lib().dw_attn_fwd_varlen_ext(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o),
                                                     _hip.ptr(lse), _hip.ptr(cu_q), _hip.ptr(cu_k), B, int(max_sq),
                                                     total_q, total_k, H, HKV, D, _row_strides(q, k, v, o),
                                                     int(causal), float(scale), ctypes.byref(args), _hip.stream()),
                   "attn_fwd_varlen_ext")
        ctx.save_for_backward(q, k, v, o, lse, cu_q, cu_k, alibi)
        ctx.meta = (int(max_sq), int(max_sk), bool(causal), float(scale), tuple(window), float(p_drop), seed)
        ctx.mark_non_differentiable(lse)
        return o, lse

    @staticmethod
    def backward(ctx, do, _dlse):
        q, k, v, o, lse, cu_q, cu_k, alibi = ctx.saved_tensors
        max_sq, max_sk, causal, scale, window, p_drop, seed = ctx.meta
        do = _rows_dense(do.to(torch.bfloat16))
        total_q, H, D = q.shape
        total_k, HKV = k.shape[0], k.shape[1]
        B = cu_q.numel() - 1
        L = _hip.lib()
        ws = torch.empty(L.dw_attn_bwd_workspace(B, max(max_sq, max_sk), H, D), device=q.device, dtype=torch.uint8)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        args = _ext_args(None, None, alibi, window, p_drop, seed)
        _hip.check(L.dw_attn_bwd_varlen_ext(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(do),
                                            _hip.ptr(lse), _hip.ptr(dq), _hip.ptr(dk), _hip.ptr(dv), _hip.ptr(ws),
                                            _hip.ptr(cu_q), _hip.ptr(cu_k), B, max_sq, max_sk, total_q, total_k, H,
                                            HKV, D, _row_strides(q, k, v, o, do, dq, dk, dv), int(causal),
                                            float(scale), ctypes.byref(args), _hip.stream()), "attn_bwd_varlen_ext")
        return dq, dk, dv, None, None, None, None, None, None, None, None, None, None


def flash_attn_varlen_func(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p=0.0,
                           softmax_scale=None, causal=False, window_size=(-1, -1), alibi_slopes=None,
                           deterministic=False, return_attn_probs=False, dropout_seed=None):
    """flash-attn's ``flash_attn_varlen_func``: q [total_q, H, D], k/v
    [total_k, Hkv, D], cu_seqlens int32 [B+1] -> [total_q, H, D]
    (``return_attn_probs``: (out, softmax_lse [H, total_q], None)).
    (Reference use: atorch/atorch/modules/transformer/layers.py:1226-1244.)"""
    D = q.shape[-1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    window = tuple(int(w) for w in window_size)
    ext = dropout_p > 0.0 or window != (-1, -1) or alibi_slopes is not None or return_attn_probs
    if _hip.bf16_path(q):
        q, k, v = _hip.bf16(q, k, v)
        if not ext:
            return _FlashAttnVarlenFn.apply(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, causal,
                                            scale)
        B = cu_seqlens_q.numel() - 1
        alibi = _prep_alibi(alibi_slopes, B, q.shape[1], q.device)
        seed = (dropout_seed if dropout_seed is not None else _new_seed()) if dropout_p > 0.0 else 0
        o, lse = _FlashAttnVarlenExtFn.apply(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, causal,
                                             scale, window, alibi, float(dropout_p), seed)
        return (o, lse, None) if return_attn_probs else o
    if dropout_p > 0.0 or window != (-1, -1) or alibi_slopes is not None:
        # CPU: per-sequence dense reference with the same masks
        cq, ck = cu_seqlens_q.tolist(), cu_seqlens_k.tolist()
        out = torch.zeros(q.shape, dtype=q.dtype, device=q.device)
        for b in range(len(cq) - 1):
            if cq[b + 1] == cq[b]:
                continue
            sl = alibi_slopes[b] if alibi_slopes is not None and alibi_slopes.dim() == 2 else alibi_slopes
            qs, ks, vs = q[cq[b]:cq[b + 1]][None], k[ck[b]:ck[b + 1]][None], v[ck[b]:ck[b + 1]][None]
            keep = (torch.rand(1, q.shape[1], qs.shape[1], ks.shape[1]) >= dropout_p) if dropout_p > 0 else None
            out[cq[b]:cq[b + 1]] = attention_reference_ext(qs, ks, vs, causal, scale, window, None, None, sl,
                                                           dropout_p, keep)[0]
        return (out, None, None) if return_attn_probs else out
    o = varlen_attention_reference(q, k, v, cu_seqlens_q, cu_seqlens_k, causal, scale)
    return (o, None, None) if return_attn_probs else o


def unpad_input(hidden: torch.Tensor, attention_mask: torch.Tensor):
    """flash-attn ``bert_padding.unpad_input``: hidden [B, S, ...], mask
    [B, S] (1 = token) -> (hidden[valid] [total, ...], indices, cu_seqlens
    int32 [B+1], max_seqlen)."""
    seqlens = attention_mask.sum(dim=-1, dtype=torch.int32)
    indices = torch.nonzero(attention_mask.flatten(), as_tuple=False).flatten()
    cu = torch.zeros(seqlens.numel() + 1, dtype=torch.int32, device=hidden.device)
    cu[1:] = torch.cumsum(seqlens, dim=0)
    flat = hidden.reshape(hidden.shape[0] * hidden.shape[1], *hidden.shape[2:])
    return flat.index_select(0, indices), indices, cu, int(seqlens.max()) if seqlens.numel() else 0


def pad_input(hidden: torch.Tensor, indices: torch.Tensor, batch: int, seqlen: int) -> torch.Tensor:
    """Inverse of :func:`unpad_input` (padding positions are zero)."""
    out = torch.zeros(batch * seqlen, *hidden.shape[1:], device=hidden.device, dtype=hidden.dtype)
    out.index_copy_(0, indices, hidden)
    return out.view(batch, seqlen, *hidden.shape[1:])


def flash_attn_padded_func(q, k, v, key_padding_mask: torch.Tensor, causal: bool = True, softmax_scale=None,
                           dropout_p: float = 0.0, window_size=(-1, -1)):
    """BSHD attention of a padded batch (``key_padding_mask`` [B, S], True =
    token, left or right padding): unpad -> varlen kernels -> pad.  Padded
    query rows return zeros."""
    B, S = q.shape[0], q.shape[1]
    qu, idx, cu, mx = unpad_input(q, key_padding_mask)
    ku = k.reshape(B * S, *k.shape[2:]).index_select(0, idx)
    vu = v.reshape(B * S, *v.shape[2:]).index_select(0, idx)
    o = flash_attn_varlen_func(qu, ku, vu, cu, cu, mx, mx, dropout_p=dropout_p, softmax_scale=softmax_scale,
                               causal=causal, window_size=window_size)
    return pad_input(o, idx, B, S)


# ------------------------------------------------------------------ decode
_DEC_WS = {}


def decode_attention_reference(q, k_cache, v_cache, lens, softmax_scale=None):
    """q [B, H, D], caches [B, Smax, Hkv, D], lens [B] -> [B, H, D] (fp32 math)."""
    B, H, D = q.shape
    hkv = k_cache.shape[2]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    out = torch.empty_like(q)
    for b in range(B):
        n = int(lens[b])
        k = k_cache[b, :n].float().repeat_interleave(H // hkv, dim=1)  # [n, H, D]
        v = v_cache[b, :n].float().repeat_interleave(H // hkv, dim=1)
        s = torch.einsum("hd,nhd->hn", q[b].float(), k) * scale
        out[b] = torch.einsum("hn,nhd->hd", s.softmax(-1), v).to(q.dtype)
    return out


def decode_attention(q, k_cache, v_cache, lens, softmax_scale=None, chunk: int = 256):
    """One-token-per-sequence attention over a static KV cache.

    q [B, H, D]; k_cache / v_cache [B, Smax, Hkv, D] (row-contiguous heads,
    any batch / row stride); lens [B] int32 on the device (valid keys per
    sequence).  The launch depends only on Smax, so a decode step can be
    captured once in a HIP graph and replayed while ``lens`` grows
    (``csrc/kernels/attn_decode.hip``: split-KV, HBM-bound)."""
    if not _hip.use_hip(q):
        return decode_attention_reference(q, k_cache, v_cache, lens, softmax_scale)
    _hip.require_bf16(q, k_cache, v_cache)
    B, H, D = q.shape
    Smax, hkv = k_cache.shape[1], k_cache.shape[2]
    if D not in (64, 128) or H % hkv or k_cache.stride(3) != 1 or k_cache.stride(2) != D or \
            v_cache.stride(3) != 1 or v_cache.stride(2) != D or lens.dtype != torch.int32 or lens.numel() != B \
            or lens.device != q.device:
        raise _hip.HipKernelError("decode_attention: bf16 q [B,H,D], caches [B,S,Hkv,D] with D in {64,128}, "
                                  "int32 device lens [B]")
    q = q.contiguous()
    nsplit = (Smax + chunk - 1) // chunk
    key = (q.device, B, H, D, nsplit)
    ws = _DEC_WS.get(key)
    if ws is None:
        ws = (torch.empty(B * H * nsplit * D, device=q.device, dtype=torch.float32),
              torch.empty(B * H * nsplit * 2, device=q.device, dtype=torch.float32))
        _DEC_WS[key] = ws
    out = torch.empty_like(q)
    st = (ctypes.c_longlong * 6)(q.stride(0), k_cache.stride(0), k_cache.stride(1), v_cache.stride(0),
                                 v_cache.stride(1), out.stride(0))
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    _hip.check(_hip.lib().dw_attn_decode(_hip.ptr(q), _hip.ptr(k_cache), _hip.ptr(v_cache), _hip.ptr(lens),
                                         _hip.ptr(out), _hip.ptr(ws[0]), _hip.ptr(ws[1]), B, H, hkv, D, nsplit,
                                         chunk, st, ctypes.c_float(scale), _hip.stream()), "attn_decode")
    return out
