"""Linear layer whose backward writes straight into flat gradient buffers.

Forward: one hipBLASLt GEMM (+ bias epilogue) via ``F.linear``.  Backward:
``dX = dY W`` (GEMM), ``dW += dY^T X`` as ``grad.addmm_`` (beta = 1: the
accumulate is the GEMM epilogue, no separate ``grad += g`` pass, no
temporary ``g``) and ``db += colsum(dY)`` with the column-reduction kernel
(``colred.hip``), when the parameters live in a ``FlatParams`` buffer with
direct gradients (see ``_grad.py``).  Otherwise plain autograd semantics.
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _hip
from ._grad import direct_grad, notify


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.weight_param, ctx.bias_param = weight, bias
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        N, K = w.shape
        dy2 = dy.reshape(-1, N)
        x2 = x.reshape(-1, K)
        dx = (dy2 @ w).view(x.shape) if ctx.needs_input_grad[0] else None
        dw = db = None
        b = ctx.bias_param
        gw = direct_grad(ctx.weight_param)
        gb = direct_grad(b) if b is not None else None
        if ctx.needs_input_grad[1]:
            if gw is not None:
                gw.addmm_(dy2.t(), x2)
                notify(ctx.weight_param)
            else:
                dw = dy2.t() @ x2
        if b is not None and ctx.needs_input_grad[2]:
            if gb is not None and _hip.use_hip(dy2) and dy2.is_contiguous() and N % 8 == 0:
                from .activation import colsum

                colsum(dy2, out=gb, accumulate=True)
                notify(b)
            else:
                db = dy2.sum(0).to(b.dtype)
        return dx, dw, db


def linear(x, weight, bias=None):
    if _hip.use_hip(x) and (getattr(weight, "_dwamd_direct", False)):
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class FusedLinear(nn.Linear):
    """``nn.Linear`` with direct flat-gradient accumulation in backward."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)
