"""Weighted Sharpness-Aware Minimization (WSAM, KDD'23).

Two forward/backward passes per step: the first gradient g0 moves the
weights to ``w + e(w)`` (e = rho * g0 / ||g0||, optionally scaled by |w|
for adaptive SAM); the gradient there, g1, defines the sharpness
``g1 - g0``.  Coupled: the base optimizer steps on
``alpha * g1 + (1 - alpha) * g0``; decoupled (default): it steps on g0 and
the sharpness is applied separately, ``w -= lr * alpha * (g1 - g0)``, with
``alpha = gamma / (1 - gamma)``.  The per-parameter work uses ``torch._foreach``
ops (one kernel per op across all parameters instead of one per tensor).

Parity: ATorch ``atorch/optimizers/wsam.py`` (``WeightedSAM``: rho, gamma,
sam_eps, adaptive, decouple, max_norm; ``first_step`` / ``second_step`` /
``step(closure)``).
"""

import torch
import torch.distributed as dist


def _bn_momentum(model, enable: bool):
    for m in model.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            if enable:
                if hasattr(m, "backup_momentum"):
                    m.momentum = m.backup_momentum
            else:
                m.backup_momentum = m.momentum
                m.momentum = 0


class WeightedSAM(torch.optim.Optimizer):
    def __init__(self, model, base_optimizer, rho=0.05, gamma=0.9, sam_eps=1e-12, adaptive=False, decouple=True,
                 max_norm=None, **kwargs):
        assert rho >= 0.0, f"invalid rho {rho}"
        self.model = model
        self.base_optimizer = base_optimizer
        self.decouple = decouple
        self.max_norm = max_norm
        alpha = gamma / (1 - gamma)
        defaults = dict(rho=rho, alpha=alpha, sam_eps=sam_eps, adaptive=adaptive, **kwargs)
        defaults.update(base_optimizer.defaults)
        super().__init__(base_optimizer.param_groups, defaults)

    def _params(self, group):
        return [p for p in group["params"] if p.grad is not None]

    @staticmethod
    def _avg_grads(ps):
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1 and ps:
            flat = torch.cat([p.grad.reshape(-1) for p in ps])
            dist.all_reduce(flat)
            flat.div_(dist.get_world_size())
            o = 0
            for p in ps:
                p.grad.copy_(flat[o:o + p.numel()].view_as(p.grad))
                o += p.numel()

    @torch.no_grad()
    def _grad_norm(self):
        norms = []
        for group in self.param_groups:
            ps = self._params(group)
            if not ps:
                continue
            gs = [g for g in (torch._foreach_mul([p.grad for p in ps], [p.abs() for p in ps])
                              if group["adaptive"] else [p.grad for p in ps])]
            norms.extend(torch._foreach_norm(gs))
        return torch.norm(torch.stack(norms)) if norms else torch.zeros(())

    @torch.no_grad()
    def first_step(self, zero_grad=False):
        # writes the parameters outside step(): order after any overlapped
        # flash-checkpoint snapshot still reading them
        from ..flash_checkpoint.copier import fence_all

        fence_all()
        gnorm = self._grad_norm()
        for group in self.param_groups:
            ps = self._params(group)
            if not ps:
                continue
            scale = group["rho"] / (gnorm + group["sam_eps"])
            e_w = torch._foreach_mul([p.grad for p in ps], scale)
            if group["adaptive"]:
                torch._foreach_mul_(e_w, torch._foreach_mul([p for p in ps], [p for p in ps]))
            torch._foreach_add_(ps, e_w)  # climb to w + e(w)
            for p, e in zip(ps, e_w):
                self.state[p]["e_w"] = e
            self._avg_grads(ps)
        if self.max_norm is not None:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.max_norm)
        for group in self.param_groups:
            for p in self._params(group):
                self.state[p]["grad"] = p.grad.detach().clone()
        if zero_grad:
            self.zero_grad()

    @torch.no_grad()
    def second_step(self, zero_grad=False):
        for group in self.param_groups:
            ps = self._params(group)
            self._avg_grads(ps)
            if ps:
                torch._foreach_sub_(ps, [self.state[p]["e_w"] for p in ps])  # back to w
        if self.max_norm is not None:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.max_norm)
        for group in self.param_groups:
            ps = self._params(group)
            if not ps:
                continue
            g0 = [self.state[p]["grad"] for p in ps]
            g1 = [p.grad for p in ps]
            if not self.decouple:
                torch._foreach_mul_(g1, group["alpha"])
                torch._foreach_add_(g1, g0, alpha=1.0 - group["alpha"])
            else:
                sharp = torch._foreach_sub(g1, g0)
                for p, s in zip(ps, sharp):
                    self.state[p]["sharpness"] = s
                for g, g_0 in zip(g1, g0):
                    g.copy_(g_0)
        self.base_optimizer.step()
        if self.decouple:
            for group in self.param_groups:
                ps = self._params(group)
                if ps:
                    torch._foreach_add_(ps, [self.state[p]["sharpness"] for p in ps],
                                        alpha=-group["lr"] * group["alpha"])
        if zero_grad:
            self.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        assert closure is not None, "WSAM needs a closure doing a full forward + backward"
        closure = torch.enable_grad()(closure)
        _bn_momentum(self.model, True)
        loss = closure()
        self.first_step(zero_grad=True)
        _bn_momentum(self.model, False)
        closure()
        self.second_step()
        return loss
