"""AGD optimizer (per-parameter PyTorch form).

AGD: an Auto-switchable optimizer using stepwise Gradient Difference as the
preconditioner (Yue et al., NeurIPS 2023).  Same hyper-parameters and update
rule as reference ``atorch/atorch/optimizers/agd.py`` (including the
``amsgrad`` / ``win`` variants and the update clip); for flat-buffer training
use :class:`dlrover_wuqiong_amd.optimizers.fused.FusedAGD` (one HIP launch).
"""

import math

import torch


class AGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), delta=1e-5, weight_decay=0.0,
                 weight_decouple=True, fixed_decay=False, amsgrad=False, win=False, clip=None):
        if lr <= 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if delta < 0.0:
            raise ValueError(f"Invalid delta value: {delta}")
        for b in betas:
            if not 0.0 <= b < 1.0:
                raise ValueError(f"Invalid beta parameter: {b}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        super().__init__(params, dict(lr=lr, betas=betas, delta=delta, weight_decay=weight_decay,
                                      weight_decouple=weight_decouple, fixed_decay=fixed_decay,
                                      amsgrad=amsgrad, win=win, clip=clip))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for grp in self.param_groups:
            b1, b2 = grp["betas"]
            lr, wd = grp["lr"], grp["weight_decay"]
            for p in grp["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse:
                    raise RuntimeError("AGD does not support sparse gradients")
                if not grp["win"]:
                    if grp["weight_decouple"]:
                        p.mul_(1.0 - (wd if grp["fixed_decay"] else lr * wd))
                    elif wd != 0:
                        g = g.add(p, alpha=wd)
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), device=p.device)
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                    if grp["amsgrad"]:
                        st["max_exp_avg_sq"] = torch.zeros_like(p)
                    if grp["win"]:
                        st["z"] = torch.zeros_like(p)
                st["step"] += 1
                t = float(st["step"])
                m, v = st["exp_avg"], st["exp_avg_sq"]
                bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
                if t == 1:
                    m.mul_(b1).add_(g, alpha=1 - b1)
                    diff = m / bc1
                else:
                    prev = m / (1 - b1 ** (t - 1))
                    m.mul_(b1).add_(g, alpha=1 - b1)
                    diff = m / bc1 - prev
                v.mul_(b2).addcmul_(diff, diff, value=1 - b2)
                if grp["amsgrad"]:
                    torch.maximum(st["max_exp_avg_sq"], v, out=st["max_exp_avg_sq"])
                    den = st["max_exp_avg_sq"].sqrt()
                else:
                    den = v.sqrt()
                den.clamp_(min=grp["delta"] * math.sqrt(bc2))
                step_size = lr * math.sqrt(bc2) / bc1
                upd = m / den
                if grp["clip"] is not None:
                    upd.clamp_(-grp["clip"], grp["clip"])
                if not grp["win"]:
                    p.add_(upd, alpha=-step_size)
                else:
                    z = st["z"]
                    z.add_(upd, alpha=-step_size).mul_(1.0 / (1.0 + wd * step_size))
                    two = 2 * step_size
                    tau = 1.0 / (3.0 + two * wd)
                    p.mul_(tau).add_(upd, alpha=-tau * two).add_(z, alpha=2 * tau)
        return loss
