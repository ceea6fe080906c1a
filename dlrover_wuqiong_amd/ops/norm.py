"""Fused LayerNorm / RMSNorm (HIP kernels in ``csrc/kernels/norm.hip``).

Parity: reference ``atorch/atorch/normalization/layernorm.py``
(``AtorchLayerNorm``) and the RMSNorm of its Llama modules.
"""

import ctypes
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _hip
from ._grad import claim, claim_all, direct_grad, notify

_FOLD = os.environ.get("DWAMD_NORM_FOLD_BIAS", "1") != "0"


def _fold_target(res, H):
    """The producer of an add-norm's residual input whose output bias
    gradient this norm's backward can take over: a fused Linear / MLP node
    (``ctx.out_bias``) whose bias accumulates into flat gradient storage.
    d(bias) = column sums of d(res) = of the norm's dx, which the small-H
    backward kernel reduces anyway -- one fewer pass over [rows, H]."""
    if not _FOLD or H >= 2048 or H % 8:
        return None
    node = getattr(res, "grad_fn", None)
    b = getattr(node, "out_bias", None)
    if b is None or direct_grad(b) is None:
        return None
    return (node, b)


def _norm_backward(ctx, dy, dres):
    """Shared backward of the plain and the fused add+norm functions: dx
    (+ dres, the residual-stream gradient, fused into the same row pass) and
    dgamma/dbeta accumulated directly into flat gradient storage if present."""
    x2, weight, mean, rstd = ctx.saved_tensors
    H = x2.shape[-1]
    R = x2.shape[0]
    dy2 = dy.contiguous().view(-1, H)
    if dy2.dtype != torch.bfloat16:
        dy2 = dy2.to(torch.bfloat16)
    if dres is not None:
        dres = dres.contiguous().view(-1, H)
        if dres.dtype != torch.bfloat16:
            dres = dres.to(torch.bfloat16)
    # sums + strip counters (of the 512-column fused path and of the small-H colsum)
    ws = _hip.zeroed_workspace(3 * H + max((H + 511) // 512, (3 * H + 255) // 256), x2.device)
    dx = torch.empty_like(x2)
    wp, bp = ctx.weight_param, ctx.bias_param
    gd, bd = direct_grad(wp), direct_grad(bp) if ctx.has_bias else None
    direct = gd is not None and (not ctx.has_bias or bd is not None)
    if direct:
        dgamma, dbeta = gd, bd
    else:
        dgamma = torch.empty(H, device=x2.device, dtype=weight.dtype)
        dbeta = torch.empty(H, device=x2.device, dtype=weight.dtype) if ctx.has_bias else None
    # the residual producer's bias gradient (ops/linear.py out_bias): same
    # flags as dgamma (accumulated into direct storage of the same dtype)
    fold = getattr(ctx, "fold", None)
    dsum = direct_grad(fold[1]) if (fold is not None and direct) else None
    if dsum is not None and dsum.dtype != dgamma.dtype:
        dsum = None
    # H <= 4096: the one-pass kernels write per-block fp32 dgamma/dbeta (/dsum)
    # partials here (2 rows per block-step at H >= 2048)
    nparts = min(512, (R + 1) // 2) * (3 if dsum is not None else 2) * H if H <= 4096 else 0
    part = torch.empty(nparts, device=x2.device, dtype=torch.float32) if nparts else None
    done = ctypes.c_int(0)
    # flags: bit 0 accumulate dgamma / dbeta (direct storage already holding
    # this step's contributions), bit 1 overwrite dsum (first contribution to
    # the producer's bias since a lazy zero_grad -- parallel/flat.py)
    acc = int(direct and not claim_all(wp, bp if ctx.has_bias else None))
    dsum_fresh = dsum is not None and claim(fold[1])
    _hip.check(_hip.lib().dw_norm_bwd3(_hip.ptr(dy2), _hip.ptr(x2), _hip.ptr(weight), _hip.ptr(mean),
                                       _hip.ptr(rstd), _hip.ptr(dres), _hip.ptr(dx), _hip.ptr(dgamma),
                                       _hip.ptr(dbeta), _hip.ptr(ws), _hip.ptr(part), nparts, R, H,
                                       int(ctx.rms), int(dgamma.dtype == torch.float32), acc | (2 * dsum_fresh),
                                       _hip.ptr(dsum), ctypes.byref(done), _hip.stream(),
                                       _hip.det_scratch(R, H, 2, x2.device)), "norm_bwd")
    if dsum_fresh and not done.value:
        dsum.zero_()  # claimed but not taken over: the producer's backward accumulates into it
    if done.value:
        fold[0].out_bias_folded = True  # the producer's backward (later) skips its own reduction
        notify(fold[1])
    if direct:
        notify(wp)
        notify(bp)
        return dx.view(dy.shape), None, None
    return dx.view(dy.shape), dgamma, dbeta


def _save(ctx, x2, weight, bias, mean, rstd, rms):
    ctx.save_for_backward(x2, weight, mean, rstd)
    ctx.rms = rms
    ctx.has_bias = bias is not None and bias.requires_grad
    ctx.weight_param, ctx.bias_param = weight, (bias if ctx.has_bias else None)


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, rms):
        H = x.shape[-1]
        x2 = x.contiguous().view(-1, H)
        R = x2.shape[0]
        _hip.require_bf16(x2, weight, bias)
        y = torch.empty_like(x2)
        mean = None if rms else torch.empty(R, device=x.device, dtype=torch.float32)
        rstd = torch.empty(R, device=x.device, dtype=torch.float32)
        _hip.check(_hip.lib().dw_norm_fwd(_hip.ptr(x2), _hip.ptr(weight), _hip.ptr(bias), _hip.ptr(y),
                                          _hip.ptr(mean), _hip.ptr(rstd), R, H, float(eps), int(rms),
                                          _hip.stream()), "norm_fwd")
        _save(ctx, x2, weight, bias, mean, rstd, rms)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        dx, dgamma, dbeta = _norm_backward(ctx, dy, None)
        return dx, dgamma, dbeta, None, None


class _AddNormFn(torch.autograd.Function):
    """(y, h) = (norm(x + res), x + res): the pre-norm residual add fused into
    the norm.  Backward: dh = norm_bwd(dy) + dh_out in one row pass; x and
    res receive the same gradient."""

    @staticmethod
    def forward(ctx, x, res, weight, bias, eps, rms, fold=None):
        ctx.fold = fold
        H = x.shape[-1]
        x2 = x.contiguous().view(-1, H)
        r2 = res.contiguous().view(-1, H)
        R = x2.shape[0]
        _hip.require_bf16(x2, r2, weight, bias)
        y = torch.empty_like(x2)
        h = torch.empty_like(x2)
        mean = None if rms else torch.empty(R, device=x.device, dtype=torch.float32)
        rstd = torch.empty(R, device=x.device, dtype=torch.float32)
        _hip.check(_hip.lib().dw_add_norm_fwd(_hip.ptr(x2), _hip.ptr(r2), _hip.ptr(weight), _hip.ptr(bias),
                                              _hip.ptr(y), _hip.ptr(h), _hip.ptr(mean), _hip.ptr(rstd), R, H,
                                              float(eps), int(rms), _hip.stream()), "add_norm_fwd")
        _save(ctx, h, weight, bias, mean, rstd, rms)
        return y.view(x.shape), h.view(x.shape)

    @staticmethod
    def backward(ctx, dy, dh):
        dx, dgamma, dbeta = _norm_backward(ctx, dy, dh)
        return dx, dx, dgamma, dbeta, None, None, None


def add_layer_norm(x, res, weight, bias, eps: float = 1e-5):
    """Returns (layer_norm(x + res), x + res)."""
    if _hip.bf16_path(x):
        x, res, weight, bias = _hip.bf16(x, res, weight, bias)
        return _AddNormFn.apply(x, res, weight, bias, eps, False, _fold_target(res, x.shape[-1]))
    h = x + res
    return F.layer_norm(h, (h.shape[-1],), weight, bias, eps), h


def add_rms_norm(x, res, weight, eps: float = 1e-6):
    """Returns (rms_norm(x + res), x + res)."""
    if _hip.bf16_path(x):
        x, res, weight = _hip.bf16(x, res, weight)
        return _AddNormFn.apply(x, res, weight, None, eps, True, _fold_target(res, x.shape[-1]))
    h = x + res
    return rms_norm(h, weight, eps), h


def layer_norm(x, weight, bias, eps: float = 1e-5):
    if _hip.bf16_path(x):
        return _NormFn.apply(*_hip.bf16(x, weight, bias), eps, False)
    return F.layer_norm(x, (x.shape[-1],), weight, bias, eps)


def rms_norm(x, weight, eps: float = 1e-6):
    if _hip.bf16_path(x):
        return _NormFn.apply(*_hip.bf16(x, weight), None, eps, True)
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * weight.float()).to(x.dtype)


class LayerNorm(nn.Module):
    """Drop-in for ``nn.LayerNorm`` (last-dim only) on the fused kernel."""

    def __init__(self, hidden, eps=1e-5, bias=True, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.zeros(hidden, device=device, dtype=dtype)) if bias else None

    def forward(self, x, res=None):
        """norm(x); with ``res``: (norm(x + res), x + res), the residual add
        fused in (``add_forward``)."""
        if res is not None:
            return self._add_forward(x, res)
        if self.bias is None and _hip.bf16_path(x):
            w = _hip.bf16(self.weight)
            return _NormFn.apply(_hip.bf16(x), w, torch.zeros_like(w), self.eps, False)
        return layer_norm(x, self.weight, self.bias, self.eps)

    def add_forward(self, x, res):
        """(norm(x + res), x + res) with the residual add fused in.  Goes
        through ``__call__`` so module hooks see the parameter use (e.g. the
        overlapped optimizer update's per-module waits)."""
        return self(x, res)

    def _add_forward(self, x, res):
        if self.bias is None and _hip.bf16_path(x):
            w = _hip.bf16(self.weight)
            x, res = _hip.bf16(x, res)
            return _AddNormFn.apply(x, res, w, torch.zeros_like(w), self.eps, False, _fold_target(res, x.shape[-1]))
        return add_layer_norm(x, res, self.weight, self.bias, self.eps)


class RMSNorm(nn.Module):
    def __init__(self, hidden, eps=1e-6, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden, device=device, dtype=dtype))

    def forward(self, x, res=None):
        if res is not None:
            return add_rms_norm(x, res, self.weight, self.eps)
        return rms_norm(x, self.weight, self.eps)

    def add_forward(self, x, res):
        return self(x, res)  # through __call__: module hooks see the parameter use


AtorchLayerNorm = LayerNorm  # reference-compatible name
