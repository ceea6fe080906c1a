"""Linear layer whose backward writes straight into flat gradient buffers.

Forward: one hipBLASLt GEMM (+ bias epilogue) via ``F.linear``.  Backward:
``dX = dY W`` (GEMM), ``dW += dY^T X`` as ``grad.addmm_`` (beta = 1: the
accumulate is the GEMM epilogue, no separate ``grad += g`` pass, no
temporary ``g``) and ``db += colsum(dY)`` with the column-reduction kernel
(``colred.hip``), when the parameters live in a ``FlatParams`` buffer with
direct gradients (see ``_grad.py``).  Otherwise plain autograd semantics.
"""

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _hip
from ._grad import claim, direct_grad, notify

# dX = dY W (dgrad) and dW += dY^T X (wgrad) are independent GEMMs;
# DWAMD_WGRAD_STREAM=1 runs the wgrad (+ bias colsum) on a per-device side
# stream concurrently with the dgrad, joined before this node's backward
# returns.  Off by default: measured on the GPT2-1.5B step it is SLOWER
# (117.4 vs 115.4 ms -- two full-chip hipBLASLt GEMMs contend for CUs and L2
# rather than filling each other's tail waves).
_WGRAD_STREAM = os.environ.get("DWAMD_WGRAD_STREAM", "0") == "1"
_SIDE = {}
# The bias gradient as the wgrad GEMM's hipBLASLt BGRADB epilogue (one pass
# over dY fewer); per shape it falls back to the column-sum kernel when the
# library has no algorithm.  Opt-in (DWAMD_WGRAD_BGRAD=1): on gfx950 / ROCm
# 7.2 the only BGRADB solutions are 32x32-tile kernels -- GPT2-1.5B's qkv
# wgrad 1013 us vs ~100 us plain + 19 us column sum, step 159 vs 116 ms
# (profiles/r4/wgrad_bgradb_ab.md)
_WGRAD_BGRAD = os.environ.get("DWAMD_WGRAD_BGRAD", "0") == "1"
_EPI_UNSUPPORTED = -100
_BGRAD_OFF = set()  # (M, K, N) without an algorithm


def _side_stream(device) -> torch.cuda.Stream:
    s = _SIDE.get(device.index)
    if s is None:
        s = _SIDE[device.index] = torch.cuda.Stream(device)
    return s


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.weight_param, ctx.bias_param = weight, bias
        # a following add-norm may take over this bias's gradient (ops/norm.py
        # _fold_target: the column sums of the residual gradient it computes
        # anyway); it sets out_bias_folded before this backward runs
        ctx.out_bias, ctx.out_bias_folded = bias, False
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        N, K = w.shape
        dy2 = dy.reshape(-1, N)
        x2 = x.reshape(-1, K)
        b = None if ctx.out_bias_folded else ctx.bias_param
        gw = direct_grad(ctx.weight_param)
        gb = direct_grad(b) if b is not None else None
        if (_WGRAD_STREAM and dy2.is_cuda and ctx.needs_input_grad[0] and ctx.needs_input_grad[1]
                and gw is not None and (b is None or gb is not None) and not torch.cuda.is_current_stream_capturing()):
            return _backward_two_streams(ctx, dy2, x2, w, x.shape, gw, gb, N)
        dx = (dy2 @ w).view(x.shape) if ctx.needs_input_grad[0] else None
        dw = db = None
        if (_WGRAD_BGRAD and gw is not None and gb is not None and ctx.needs_input_grad[1] and ctx.needs_input_grad[2]
                and _hip.use_hip(dy2) and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16
                and gw.dtype == torch.bfloat16 and dy2.is_contiguous() and x2.is_contiguous()
                and (dy2.shape[0], K, N) not in _BGRAD_OFF):
            db32 = torch.empty(N, device=dy2.device, dtype=torch.float32)
            ow = claim(ctx.weight_param)
            rc = _hip.lib().dw_gemm_wgrad_bgradb(_hip.ptr(x2), _hip.ptr(dy2), _hip.ptr(gw), _hip.ptr(db32),
                                                 dy2.shape[0], K, N, 0 if ow else 1, _hip.stream())
            if rc == _EPI_UNSUPPORTED:
                _BGRAD_OFF.add((dy2.shape[0], K, N))
                if ow:
                    gw.zero_()  # claimed: the fallback below accumulates
            else:
                _hip.check(rc, "gemm_wgrad_bgradb")
                gb.copy_(db32) if claim(b) else gb.add_(db32)
                notify(ctx.weight_param)
                notify(b)
                return dx, None, None
        if ctx.needs_input_grad[1]:
            if gw is not None:
                _wgrad(gw, dy2, x2, ctx.weight_param)
                notify(ctx.weight_param)
            else:
                dw = dy2.t() @ x2
        if b is not None and ctx.needs_input_grad[2]:
            if gb is not None and _hip.use_hip(dy2) and dy2.is_contiguous() and N % 8 == 0:
                from .activation import colsum

                colsum(dy2, out=gb, accumulate=not claim(b))
                notify(b)
            else:
                db = dy2.sum(0).to(b.dtype)
        return dx, dw, db


def _wgrad(gw, dy2, x2, param):
    """gw (+)= dy2^T x2: overwrite (GEMM beta = 0) on the parameter's first
    contribution since a lazy zero_grad, else accumulate (beta = 1)."""
    if claim(param):
        torch.mm(dy2.t(), x2, out=gw)
    else:
        gw.addmm_(dy2.t(), x2)


def _backward_two_streams(ctx, dy2, x2, w, x_shape, gw, gb, N):
    """dgrad on the current stream, wgrad (+ bias colsum) on the side stream,
    both into direct flat-gradient storage; joined before returning."""
    cur = torch.cuda.current_stream(dy2.device)
    side = _side_stream(dy2.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        _wgrad(gw, dy2, x2, ctx.weight_param)
        if gb is not None:
            if _hip.use_hip(dy2) and dy2.is_contiguous() and N % 8 == 0:
                from .activation import colsum

                colsum(dy2, out=gb, accumulate=not claim(ctx.bias_param))
            elif claim(ctx.bias_param):
                gb.copy_(dy2.sum(0).to(gb.dtype))
            else:
                gb.add_(dy2.sum(0).to(gb.dtype))
    dx = (dy2 @ w).view(x_shape)
    # join: everything the caller's stream does next -- including freeing dy2
    # / x2 for reuse -- is ordered after the wgrad (no record_stream needed)
    cur.wait_stream(side)
    notify(ctx.weight_param)
    if gb is not None:
        notify(ctx.bias_param)
    return dx, None, None


def linear(x, weight, bias=None):
    if _hip.use_hip(x) and (getattr(weight, "_dwamd_direct", False)):
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class FusedLinear(nn.Linear):
    """``nn.Linear`` with direct flat-gradient accumulation in backward."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)
