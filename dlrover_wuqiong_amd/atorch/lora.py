"""Low-rank adaptation (LoRA) of linear layers (reference:
examples/pytorch/nanogpt/lora.py ``apply_lora`` / ``merge_lora``, and the
PEFT paths of AtorchTrainer).

The reference re-parametrises the weight (W + s·B·A materialised every
forward).  Here the adapter is a side branch: y = base(x) + s·(drop(x)·Aᵀ)·Bᵀ
-- two skinny GEMMs of rank r next to the frozen base GEMM (which keeps its
fused HIP epilogue), so a forward writes r·(in + out) extra values per token
instead of a full in×out weight, and the frozen base weight never gets a
gradient buffer.  ``merge_lora`` folds s·B·A into the base weight once for
inference / export.
"""

import math
from typing import Dict, Iterable, List, Optional

import torch
import torch.nn as nn


class LoraLinear(nn.Module):
    """Wraps a frozen ``nn.Linear`` (or ``FusedLinear``) with a rank-r adapter;
    B starts at zero, so the wrapped layer initially computes the base output."""

    def __init__(self, base: nn.Linear, rank: int = 4, alpha: float = 1.0, dropout: float = 0.0):
        super().__init__()
        if rank <= 0:
            raise ValueError("LoRA rank must be positive")
        self.base = base
        self.rank, self.alpha = rank, alpha
        self.scaling = alpha / rank
        w = base.weight
        self.lora_A = nn.Parameter(torch.empty(rank, base.in_features, device=w.device, dtype=w.dtype))
        self.lora_B = nn.Parameter(torch.zeros(base.out_features, rank, device=w.device, dtype=w.dtype))
        nn.init.kaiming_uniform_(self.lora_A, a=math.sqrt(5))
        self.dropout = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        for p in base.parameters():
            p.requires_grad_(False)
        self.merged = False
        self._register_load_state_dict_pre_hook(self._from_base_keys)

    def _from_base_keys(self, state_dict, prefix, *_args):
        # a plain (pre-LoRA) checkpoint: its weight / bias are the base
        # layer's, the adapter keeps its current (B = 0) values
        for k in ("weight", "bias"):
            if prefix + k in state_dict and prefix + "base." + k not in state_dict:
                state_dict[prefix + "base." + k] = state_dict.pop(prefix + k)
        if prefix + "base.weight" in state_dict:
            state_dict.setdefault(prefix + "lora_A", self.lora_A.detach().clone())
            state_dict.setdefault(prefix + "lora_B", self.lora_B.detach().clone())

    @property
    def weight(self):
        return self.base.weight

    @property
    def bias(self):
        return self.base.bias

    @property
    def in_features(self):
        return self.base.in_features

    @property
    def out_features(self):
        return self.base.out_features

    def forward(self, x):
        y = self.base(x)
        if self.merged:
            return y
        h = nn.functional.linear(self.dropout(x).to(self.lora_A.dtype), self.lora_A)
        return y + (nn.functional.linear(h, self.lora_B) * self.scaling).to(y.dtype)

    @torch.no_grad()
    def merge(self):
        """W += s·B·A (in fp32, once); the adapter branch is skipped after."""
        if not self.merged:
            delta = (self.lora_B.float() @ self.lora_A.float()) * self.scaling
            self.base.weight.add_(delta.to(self.base.weight.dtype))
            self.merged = True

    def extra_repr(self):
        return f"rank={self.rank}, alpha={self.alpha}, merged={self.merged}"


def apply_lora(model: nn.Module, targets: Optional[Iterable[str]] = None, rank: int = 4, dropout: float = 0.0,
               alpha: float = 1.0, freeze_others: bool = True) -> List[str]:
    """Wrap every ``nn.Linear`` whose qualified name contains one of
    ``targets`` (all linears when ``targets`` is empty/None) and, with
    ``freeze_others``, freeze every non-adapter parameter.  Returns the
    wrapped names."""
    targets = [t for t in (targets or []) if t]
    done = []
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            full = f"{name}.{cname}" if name else cname
            if isinstance(child, nn.Linear) and (not targets or any(t in full for t in targets)):
                setattr(mod, cname, LoraLinear(child, rank=rank, alpha=alpha, dropout=dropout))
                done.append(full)
    if freeze_others:
        for n, p in model.named_parameters():
            p.requires_grad_("lora_A" in n or "lora_B" in n)
    return done


def merge_lora(model: nn.Module) -> int:
    n = 0
    for m in model.modules():
        if isinstance(m, LoraLinear):
            m.merge()
            n += 1
    return n


def lora_state_dict(model: nn.Module) -> Dict[str, torch.Tensor]:
    """Only the adapter tensors (what a fine-tuning checkpoint needs)."""
    return {k: v for k, v in model.state_dict().items() if "lora_A" in k or "lora_B" in k}


def create_lora_config(args) -> Optional[dict]:
    """``--lora_rank/--lora_dropout/--lora_alpha/--lora_targets`` -> apply_lora kwargs
    (None when no LoRA flag is set)."""
    vals = [getattr(args, k, None) for k in ("lora_rank", "lora_dropout", "lora_alpha", "lora_targets")]
    if all(v is None for v in vals):
        return None
    rank, dropout, alpha, targets = vals
    return {"rank": rank or 4, "dropout": dropout or 0.0, "alpha": alpha or 1.0,
            "targets": targets.split(",") if isinstance(targets, str) and targets else []}


__all__ = ["LoraLinear", "apply_lora", "merge_lora", "lora_state_dict", "create_lora_config"]
