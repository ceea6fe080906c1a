"""BF16Optimizer: fp32 master weights around any optimizer for bf16 models.

The wrapped optimizer's parameter groups are re-pointed to fp32 master
copies of every bf16/fp16 parameter; ``step()`` copies the low-precision
gradients into the masters' ``.grad`` (fp32), runs the inner step on the
masters and writes them back rounded to the model dtype.  Gradients that are
not finite skip the step (``skip_if_nonfinite``), matching the reference's
overflow handling for bf16 fine-tuning.

For flat-buffer models prefer ``optimizers.fused.FusedAdamW`` (masters live
inside the fused HIP kernel, one pass over HBM); this wrapper exists for
arbitrary ``torch.optim`` optimizers and per-parameter models.

Parity: ATorch ``atorch/optimizers/bf16_optimizer.py`` (``BF16Optimizer``,
``model_grads_to_master_grads``, ``master_params_to_model_params``).
"""

from typing import Dict, List

import torch

_LOW = (torch.bfloat16, torch.float16)


def model_grads_to_master_grads(model_params: List[torch.Tensor], master_params: List[torch.Tensor]):
    for m, mp in zip(model_params, master_params):
        if m.grad is None:
            mp.grad = None
            continue
        if mp.grad is None:
            mp.grad = torch.empty_like(mp)
        mp.grad.copy_(m.grad)


def master_params_to_model_params(model_params: List[torch.Tensor], master_params: List[torch.Tensor]):
    for m, mp in zip(model_params, master_params):
        m.data.copy_(mp.data)


class BF16Optimizer(torch.optim.Optimizer):
    """``BF16Optimizer(torch.optim.AdamW(model.parameters(), lr=...))``."""

    def __init__(self, init_optimizer: torch.optim.Optimizer, skip_if_nonfinite: bool = True, verbose: bool = False):
        self.optimizer = init_optimizer
        self.skip_if_nonfinite = skip_if_nonfinite
        self.verbose = verbose
        self.low_groups: List[List[torch.Tensor]] = []
        self.master_groups: List[List[torch.Tensor]] = []
        self.fp32_groups: List[List[torch.Tensor]] = []
        self.skipped_steps = 0
        for group in self.optimizer.param_groups:
            lows, masters, fp32s = [], [], []
            for i, p in enumerate(group["params"]):
                if not p.requires_grad:
                    continue
                if p.dtype in _LOW:
                    mp = p.detach().clone().float()
                    mp.requires_grad_(True)
                    group["params"][i] = mp
                    if p in self.optimizer.state:
                        self.optimizer.state[mp] = self.optimizer.state.pop(p)
                    lows.append(p)
                    masters.append(mp)
                elif p.dtype == torch.float32:
                    fp32s.append(p)
                else:
                    raise TypeError(f"BF16Optimizer: unsupported parameter dtype {p.dtype}")
            self.low_groups.append(lows)
            self.master_groups.append(masters)
            self.fp32_groups.append(fp32s)

    # torch.optim.Optimizer protocol ---------------------------------------------------
    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @param_groups.setter
    def param_groups(self, v):
        self.optimizer.param_groups = v

    @property
    def state(self):
        return self.optimizer.state

    @property
    def defaults(self):
        return self.optimizer.defaults

    def __getstate__(self):
        raise RuntimeError("BF16Optimizer should be serialized with state_dict()")

    def __repr__(self):
        return f"BF16Optimizer({self.optimizer!r})"

    def zero_grad(self, set_to_none: bool = True):
        for lows, masters, fp32s in zip(self.low_groups, self.master_groups, self.fp32_groups):
            for p in lows + masters + fp32s:
                if p.grad is None:
                    continue
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.detach_()
                    p.grad.zero_()

    def _grads_finite(self) -> bool:
        norms = []
        for lows, fp32s in zip(self.low_groups, self.fp32_groups):
            for p in lows + fp32s:
                if p.grad is not None:
                    norms.append(p.grad.detach().float().abs().amax())
        if not norms:
            return True
        return bool(torch.isfinite(torch.stack(norms)).all())

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self.skip_if_nonfinite and not self._grads_finite():
            self.skipped_steps += 1
            if self.verbose:
                print(f"BF16Optimizer: non-finite gradients, step skipped ({self.skipped_steps})")
            return loss
        for lows, masters in zip(self.low_groups, self.master_groups):
            model_grads_to_master_grads(lows, masters)
        self.optimizer.step()
        for lows, masters in zip(self.low_groups, self.master_groups):
            master_params_to_model_params(lows, masters)
        return loss

    def clip_master_grads(self, max_norm: float, norm_type: float = 2.0) -> torch.Tensor:
        """Clip the fp32 master gradients (call after ``backward``; copies the
        model gradients to the masters first)."""
        for lows, masters in zip(self.low_groups, self.master_groups):
            model_grads_to_master_grads(lows, masters)
        params = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
        total = torch.nn.utils.clip_grad_norm_(params, max_norm, norm_type)
        for lows, masters in zip(self.low_groups, self.master_groups):
            for m, mp in zip(lows, masters):
                if mp.grad is not None:
                    m.grad.copy_(mp.grad)
        return total

    def state_dict(self) -> Dict:
        return {"optimizer_state_dict": self.optimizer.state_dict(),
                "fp32_from_fp16": [[p.detach().clone() for p in g] for g in self.master_groups],
                "skipped_steps": self.skipped_steps}

    def load_state_dict(self, sd: Dict):
        self.optimizer.load_state_dict(sd["optimizer_state_dict"])
        self.skipped_steps = sd.get("skipped_steps", 0)
        for cur, saved, lows in zip(self.master_groups, sd["fp32_from_fp16"], self.low_groups):
            for mp, s, m in zip(cur, saved, lows):
                mp.data.copy_(s)
                m.data.copy_(s)
