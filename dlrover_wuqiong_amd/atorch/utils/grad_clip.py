"""Gradient-norm clipping for models returned by ``auto_accelerate`` and a
parameter counter (reference: atorch/atorch/auto/clip_grad_norm.py:13,
trainer/atorch_trainer.py ``count_model_params``).

One entry point for every wrapper this framework produces:

* FSDP2 / TP (DTensor parameters): the per-shard norms are combined by
  ``torch.nn.utils.clip_grad_norm_`` over the mesh, the returned DTensor is
  materialised with ``full_tensor()`` so every rank gets the same float;
* an optimizer that owns the gradients (flat ZeRO / BF16 master optimizers
  expose ``clip_grad_norm``) clips its own buffers;
* FSDP1-style modules that expose ``clip_grad_norm_`` use it;
* everything else (DDP, single GPU) is the plain torch clip.
"""

from typing import Optional

import torch
import torch.nn as nn


def clip_grad_norm(model: nn.Module, max_norm: float, norm_type: float = 2.0,
                   optimizer: Optional[torch.optim.Optimizer] = None, process_group_name_prefix: str = ""):
    """Clip gradients in place; returns the total (pre-clip) norm as a tensor,
    or None when no parameter has a gradient."""
    del process_group_name_prefix  # groups come from the parameters' meshes
    if optimizer is not None and callable(getattr(optimizer, "clip_grad_norm", None)):
        return optimizer.clip_grad_norm(max_norm, norm_type)
    if callable(getattr(model, "clip_grad_norm_", None)):
        return model.clip_grad_norm_(max_norm, norm_type)
    params = [p for p in model.parameters() if p.grad is not None]
    if not params:
        return None
    total = torch.nn.utils.clip_grad_norm_(params, max_norm, norm_type=norm_type)
    full = getattr(total, "full_tensor", None)
    return full() if callable(full) else total


def count_model_params(model: nn.Module, trainable_only: bool = False) -> int:
    """Global parameter count (DTensor shards counted at their full size)."""
    n = 0
    for p in model.parameters():
        if trainable_only and not p.requires_grad:
            continue
        n += p.numel()  # DTensor.numel() is the global size
    return n
