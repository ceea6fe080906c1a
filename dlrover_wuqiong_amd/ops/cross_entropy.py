"""Fused cross-entropy over large vocabularies (``csrc/kernels/xent.hip``).

Parity: reference ``atorch/atorch/modules/transformer/cross_entropy.py``
(``AtorchCrossEntropyLoss``).
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _hip


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, smoothing, reduction, inplace_grad):
        V = logits.shape[-1]
        x = logits.contiguous().view(-1, V)
        _hip.require_bf16(x)
        t = target.contiguous().view(-1).to(torch.int64)
        T = x.shape[0]
        loss = torch.empty(T, device=x.device, dtype=torch.float32)
        lse = torch.empty(T, device=x.device, dtype=torch.float32)
        _hip.check(_hip.lib().dw_xent_fwd(_hip.ptr(x), _hip.ptr(t), _hip.ptr(loss), _hip.ptr(lse), None, None,
                                          T, V, int(ignore_index), 0, float(smoothing), _hip.stream()),
                   "xent_fwd")
        ctx.save_for_backward(x, t, lse)
        ctx.meta = (ignore_index, smoothing, reduction, inplace_grad, logits.shape)
        if reduction == "none":
            return loss.view(target.shape)
        if reduction == "sum":
            return loss.sum()
        n_valid = (t != ignore_index).sum().clamp(min=1)
        ctx.n_valid = n_valid
        return loss.sum() / n_valid

    @staticmethod
    def backward(ctx, dloss):
        x, t, lse = ctx.saved_tensors
        ignore_index, smoothing, reduction, inplace_grad, shape = ctx.meta
        T, V = x.shape
        if reduction == "none":
            g = dloss.contiguous().view(-1).float()
            per_row = 1
        elif reduction == "sum":
            g = dloss.float().view(1)
            per_row = 0
        else:
            g = (dloss.float() / ctx.n_valid).view(1)
            per_row = 0
        dx = x if inplace_grad else torch.empty_like(x)
        _hip.check(_hip.lib().dw_xent_bwd(_hip.ptr(x), _hip.ptr(t), _hip.ptr(lse), _hip.ptr(g), per_row,
                                          _hip.ptr(dx), T, V, int(ignore_index), 0, float(smoothing),
                                          _hip.stream()), "xent_bwd")
        return dx.view(shape), None, None, None, None, None


def cross_entropy(logits, target, ignore_index=-100, label_smoothing=0.0, reduction="mean",
                  inplace_grad=False):
    """``inplace_grad=True`` writes dlogits over the logits buffer in the
    backward (saves T*V*2 bytes; only valid when nothing else reads the
    logits after the loss)."""
    if _hip.bf16_path(logits):
        return _XentFn.apply(_hip.bf16(logits), target, ignore_index, label_smoothing, reduction, inplace_grad)
    out = F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), target.reshape(-1),
                          ignore_index=ignore_index, label_smoothing=label_smoothing, reduction=reduction)
    return out.reshape(target.shape) if reduction == "none" else out


class CrossEntropyLoss(nn.Module):
    def __init__(self, ignore_index=-100, label_smoothing=0.0, reduction="mean"):
        super().__init__()
        self.ignore_index = ignore_index
        self.label_smoothing = label_smoothing
        self.reduction = reduction

    def forward(self, logits, target):
        return cross_entropy(logits, target, self.ignore_index, self.label_smoothing, self.reduction)


AtorchCrossEntropyLoss = CrossEntropyLoss
