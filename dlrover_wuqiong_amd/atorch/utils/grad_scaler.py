"""Grad scalers for bf16 training: no loss scaling (bf16 has fp32's
exponent range), but the step is still skipped when a gradient is inf/nan
and ``has_overflow()`` reports it -- the skip-on-overflow half of AMP
without the scale search.  ``BF16ShardedGradScaler`` does the same for
sharded (FSDP) gradients, agreeing on overflow across the process group.

Parity: ATorch ``atorch/utils/grad_scaler.py`` (BF16GradScaler,
BF16ShardedGradScaler).
"""

import torch
import torch.distributed as dist

from ...common.log import logger

try:
    from torch.amp import GradScaler as _GradScaler
except ImportError:  # pragma: no cover
    from torch.cuda.amp import GradScaler as _GradScaler


def _found_inf(optimizer_state) -> bool:
    vals = list(optimizer_state["found_inf_per_device"].values())
    return bool(vals) and float(torch.stack([v.float().to(vals[0].device) for v in vals]).sum()) > 0


class BF16GradScaler(_GradScaler):
    def __init__(self, init_scale=1.0, growth_factor=1.0, backoff_factor=1.0, growth_interval=2 ** 62, enabled=True,
                 device="cuda"):
        dev = device if torch.cuda.is_available() else "cpu"
        # torch requires growth > 1 > backoff; update() pins the scale at 1
        super().__init__(dev, init_scale=1.0, growth_factor=2.0, backoff_factor=0.5, growth_interval=2 ** 62,
                         enabled=enabled)
        self.overflow = False

    def update(self, new_scale=None):
        super().update(new_scale)
        if getattr(self, "_scale", None) is not None:
            self._scale.fill_(1.0)

    def scale(self, outputs):
        self.overflow = False
        return super().scale(outputs)

    def _maybe_opt_step(self, optimizer, optimizer_state, *args, **kwargs):
        if _found_inf(optimizer_state):
            self.overflow = True
            logger.info("BF16GradScaler: inf/nan gradient, optimizer step skipped")
            return None
        return optimizer.step(*args, **kwargs)

    def has_overflow(self) -> bool:
        return self.overflow


class BF16ShardedGradScaler(BF16GradScaler):
    """Each rank holds a gradient shard: the overflow decision is all-reduced
    (MAX) over ``process_group`` so every rank skips the same step."""

    def __init__(self, *args, process_group=None, **kwargs):
        super().__init__(*args, **kwargs)
        self.process_group = process_group

    def _maybe_opt_step(self, optimizer, optimizer_state, *args, **kwargs):
        inf = _found_inf(optimizer_state)
        if dist.is_available() and dist.is_initialized():
            dev = "cuda" if dist.get_backend(self.process_group) == "nccl" else "cpu"
            t = torch.tensor([1.0 if inf else 0.0], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.process_group)
            inf = bool(t.item() > 0)
        if inf:
            self.overflow = True
            logger.info("BF16ShardedGradScaler: inf/nan gradient on some rank, optimizer step skipped")
            return None
        return optimizer.step(*args, **kwargs)
