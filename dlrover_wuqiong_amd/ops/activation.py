"""Fused activations: bias+GeLU(tanh) and SwiGLU (``csrc/kernels/elementwise.hip``)."""

import math

import torch
import torch.nn.functional as F

from . import _hip
from ._grad import claim, direct_grad, notify


def colsum(x2: torch.Tensor, out_dtype=None, out: torch.Tensor = None, accumulate: bool = False) -> torch.Tensor:
    """Column sums of a [rows, C] bf16 tensor (bias gradients), fp32 math;
    ``out`` (+)= result when given (direct flat-gradient accumulation)."""
    R, C = x2.shape
    if out is None:
        out = torch.empty(C, device=x2.device, dtype=out_dtype or x2.dtype)
    ws = _hip.zeroed_workspace(C + (C + 511) // 512, x2.device)  # sums + strip counters
    _hip.check(_hip.lib().dw_colsum_acc(_hip.ptr(x2), R, C, _hip.ptr(ws), _hip.ptr(out),
                                        int(out.dtype == torch.float32), int(accumulate), _hip.stream(),
                                        _hip.det_scratch(R, C, 0, x2.device)), "colsum")
    return out


_colsum = colsum


class _BiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias):
        C = x.shape[-1]
        x = x.contiguous()
        _hip.require_bf16(x, bias)
        y = torch.empty_like(x)
        pre = torch.empty_like(x) if bias is not None else None
        _hip.check(_hip.lib().dw_bias_gelu_fwd(_hip.ptr(x), _hip.ptr(bias), _hip.ptr(y), _hip.ptr(pre),
                                               x.numel(), C, _hip.stream()), "bias_gelu_fwd")
        ctx.save_for_backward(pre if pre is not None else x)
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.bias_param = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        (pre,) = ctx.saved_tensors
        dy = dy.contiguous().to(torch.bfloat16)
        dx = torch.empty_like(pre)
        if not ctx.has_bias:
            _hip.check(_hip.lib().dw_gelu_bwd(_hip.ptr(dy), _hip.ptr(pre), _hip.ptr(dx), pre.numel(),
                                              _hip.stream()), "gelu_bwd")
            return dx, None
        # one pass: dx = dy * gelu'(pre) and dbias (+)= colsum(dx)
        C = pre.shape[-1]
        g = direct_grad(ctx.bias_param)
        db = g if g is not None else torch.empty(C, device=pre.device, dtype=ctx.bias_dtype)
        ws = _hip.zeroed_workspace(C + (C + 511) // 512, pre.device)
        _hip.check(_hip.lib().dw_gelu_bwd_dbias(_hip.ptr(dy), _hip.ptr(pre), _hip.ptr(dx), pre.numel() // C, C,
                                                _hip.ptr(ws), _hip.ptr(db), int(db.dtype == torch.float32),
                                                int(g is not None and not claim(ctx.bias_param)), _hip.stream(),
                                                _hip.det_scratch(pre.numel() // C, C, 1, pre.device)),
                   "gelu_bwd_dbias")
        if g is not None:
            notify(ctx.bias_param)
            return dx, None
        return dx, db


def _gelu_tanh_ref(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x.pow(3))))


def bias_gelu(x, bias=None):
    """gelu_tanh(x + bias) — GPT-2's MLP activation."""
    if _hip.bf16_path(x):
        return _BiasGeluFn.apply(*_hip.bf16(x, bias))
    y = x + bias if bias is not None else x
    return F.gelu(y, approximate="tanh")


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        _hip.require_bf16(x)
        C2 = x.shape[-1]
        C = C2 // 2
        R = x.numel() // C2
        y = torch.empty(*x.shape[:-1], C, device=x.device, dtype=x.dtype)
        _hip.check(_hip.lib().dw_swiglu_fwd(_hip.ptr(x), _hip.ptr(y), R, C, _hip.stream()), "swiglu_fwd")
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous().to(torch.bfloat16)
        C2 = x.shape[-1]
        C = C2 // 2
        R = x.numel() // C2
        dx = torch.empty_like(x)
        _hip.check(_hip.lib().dw_swiglu_bwd(_hip.ptr(dy), _hip.ptr(x), _hip.ptr(dx), R, C, _hip.stream()),
                   "swiglu_bwd")
        return dx


def swiglu(x):
    """silu(x[..., :C]) * x[..., C:] for x of last dim 2C (fused gate|up)."""
    if _hip.bf16_path(x):
        return _SwiGLUFn.apply(_hip.bf16(x))
    a, b = x.chunk(2, dim=-1)
    return F.silu(a) * b
