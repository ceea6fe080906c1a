"""Low-bit AdamW: optimizer states stored in 4 (or 8) bits per element.

``Q_AdamW(params, lr, betas, eps, weight_decay, q_bits=4, threshold=4096)``
keeps, for every parameter with at least ``threshold`` elements, the first
and second moments as block-quantized codes (groups of 128, one fp32 scale
per group) and updates them with ONE fused HIP kernel
(``csrc/kernels/optim_lowbit.hip``).  Small tensors (norms, biases) keep
fp32 states.  The quantization maps (see the kernel header) are a dense-near-
zero signed map for m and a zero-point-free quadratic map for v.

On CPU the identical algorithm runs in PyTorch (``_ref_step``), which is also
the fp32 reference the GPU test compares the kernel against.

``Q_AGD``, ``Q_Adafactor`` and ``Q_CAME`` keep their moments in the same
codec through ``QState`` (decode -> fp32 update -> encode; row/column
statistics of factored second moments stay fp32 since they are O(rows+cols)).

Parity: ATorch ``atorch/optimizers/low_bit/optim/{q_adamw,q_agd,q_adafactor,
q_came}.py`` (``q_bits``, ``threshold`` and the per-optimizer hyper-parameters).
"""

import math
from typing import Optional

import torch

GROUP = 128
M4 = torch.tensor([0.0, 0.015625, 0.0625, 0.125, 0.25, 0.5, 0.75, 1.0,
                   0.0, -0.015625, -0.0625, -0.125, -0.25, -0.5, -0.75, -1.0])
_M4_MID = torch.tensor([0.0078125, 0.0390625, 0.09375, 0.1875, 0.375, 0.625, 0.875])


def _pad(n: int) -> int:
    return (n + GROUP - 1) // GROUP * GROUP


# ------------------------------------------------------------ reference codec
def quant_m(x: torch.Tensor, bits: int):
    """x [G, 128] fp32 -> (codes uint8 [G, 128], scale [G])."""
    scale = x.abs().amax(1)
    inv = torch.where(scale > 0, 1.0 / scale, torch.zeros_like(scale))
    y = x * inv[:, None]
    if bits == 4:
        k = (y.abs()[..., None] > _M4_MID.to(x.device)).sum(-1)
        codes = torch.where((y < 0) & (k > 0), k | 8, k)
    else:
        codes = torch.round(y * 127).clamp(-127, 127).to(torch.int64) & 0xFF
    return codes.to(torch.uint8), scale


def dequant_m(codes: torch.Tensor, scale: torch.Tensor, bits: int):
    if bits == 4:
        return M4.to(codes.device)[codes.long()] * scale[:, None]
    c = codes.to(torch.int16)
    c = torch.where(c > 127, c - 256, c).float()
    return c * (scale[:, None] / 127.0)


def quant_v(v: torch.Tensor, bits: int):
    L = 16 if bits == 4 else 256
    scale = v.amax(1)
    safe = torch.where(scale > 0, scale, torch.ones_like(scale))
    k = torch.round(torch.sqrt(v / safe[:, None]) * L) - 1
    k = k.clamp(0, L - 1)
    k = torch.where(scale[:, None] > 0, k, torch.zeros_like(k))
    return k.to(torch.uint8), scale


def dequant_v(codes: torch.Tensor, scale: torch.Tensor, bits: int):
    L = 16 if bits == 4 else 256
    r = (codes.float() + 1) / L
    return r * r * scale[:, None]


def _pack4(codes: torch.Tensor) -> torch.Tensor:
    c = codes.view(-1, 2)
    return (c[:, 0] | (c[:, 1] << 4)).contiguous()


def _unpack4(packed: torch.Tensor) -> torch.Tensor:
    return torch.stack([packed & 15, packed >> 4], 1).view(-1)


class Q_AdamW(torch.optim.Optimizer):  # noqa: N801 (reference name)
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, q_bits: int = 4,
                 threshold: int = 4096, grad_scale: float = 1.0):
        if q_bits not in (4, 8):
            raise ValueError("q_bits must be 4 or 8")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, q_bits=q_bits, threshold=threshold)
        super().__init__(params, defaults)
        self.grad_scale = grad_scale

    def _init_state(self, p, group):
        st = self.state[p]
        st["step"] = 0
        n = p.numel()
        if n >= group["threshold"]:
            npad = _pad(n)
            nbytes = npad // 2 if group["q_bits"] == 4 else npad
            st["mq"] = torch.zeros(nbytes, dtype=torch.uint8, device=p.device)
            st["vq"] = torch.zeros(nbytes, dtype=torch.uint8, device=p.device)
            st["ms"] = torch.zeros(npad // GROUP, dtype=torch.float32, device=p.device)
            st["vs"] = torch.zeros(npad // GROUP, dtype=torch.float32, device=p.device)
        else:
            st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
            st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    self._init_state(p, group)
                st["step"] += 1
                t = st["step"]
                bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
                if "mq" in st:
                    if p.is_cuda and p.is_contiguous() and p.grad.is_contiguous():
                        self._hip_step(p, st, group, bc1, bc2)
                    else:
                        self._ref_step(p, st, group, bc1, bc2)
                else:
                    g = p.grad.float() * self.grad_scale
                    st["exp_avg"].mul_(b1).add_(g, alpha=1 - b1)
                    st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
                    upd = (st["exp_avg"] / bc1) / ((st["exp_avg_sq"] / bc2).sqrt() + group["eps"])
                    pf = p.float().mul_(1 - group["lr"] * group["weight_decay"]).add_(upd, alpha=-group["lr"])
                    p.copy_(pf)
        return loss

    def _hip_step(self, p, st, group, bc1, bc2):
        from ..ops import _hip

        b1, b2 = group["betas"]
        n = p.numel()
        pd = 0 if p.dtype == torch.bfloat16 else 1
        gd = 0 if p.grad.dtype == torch.bfloat16 else 1
        if p.dtype not in (torch.bfloat16, torch.float32) or p.grad.dtype not in (torch.bfloat16, torch.float32):
            return self._ref_step(p, st, group, bc1, bc2)
        _hip.check(_hip.lib().dw_qadamw(_hip.ptr(p), _hip.ptr(p.grad), _hip.ptr(st["mq"]), _hip.ptr(st["vq"]),
                                        _hip.ptr(st["ms"]), _hip.ptr(st["vs"]), n, _pad(n) // GROUP,
                                        group["q_bits"], pd, gd, float(group["lr"]), float(b1), float(b2),
                                        float(group["eps"]), float(group["weight_decay"]), float(bc1), float(bc2),
                                        float(self.grad_scale), _hip.stream()), "qadamw")

    def _ref_step(self, p, st, group, bc1, bc2):
        bits = group["q_bits"]
        b1, b2 = group["betas"]
        n = p.numel()
        npad = _pad(n)
        G = npad // GROUP
        mc = _unpack4(st["mq"]) if bits == 4 else st["mq"]
        vc = _unpack4(st["vq"]) if bits == 4 else st["vq"]
        m = dequant_m(mc.view(G, GROUP), st["ms"], bits)
        v = dequant_v(vc.view(G, GROUP), st["vs"], bits)
        m = torch.where(st["ms"][:, None] > 0, m, torch.zeros_like(m)).view(-1)
        v = torch.where(st["vs"][:, None] > 0, v, torch.zeros_like(v)).view(-1)
        g = torch.zeros(npad, device=p.device)
        g[:n] = p.grad.reshape(-1).float() * self.grad_scale
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        m[n:] = 0
        v[n:] = 0
        pf = p.reshape(-1).float()
        pf = pf * (1 - group["lr"] * group["weight_decay"]) - group["lr"] * (m[:n] / bc1) / (
            torch.sqrt(v[:n] / bc2) + group["eps"])
        p.copy_(pf.view_as(p).to(p.dtype))
        mcodes, ms = quant_m(m.view(G, GROUP), bits)
        vcodes, vs = quant_v(v.view(G, GROUP), bits)
        st["mq"].copy_(_pack4(mcodes.view(-1)) if bits == 4 else mcodes.view(-1))
        st["vq"].copy_(_pack4(vcodes.view(-1)) if bits == 4 else vcodes.view(-1))
        st["ms"].copy_(ms)
        st["vs"].copy_(vs)

    def state_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for st in self.state.values() for t in st.values()
                   if torch.is_tensor(t))


# ------------------------------------------------------------ generic quantized state
class QState:
    """One optimizer state tensor held as group-quantized codes (128 elements
    per fp32 scale).  ``signed=True`` uses the first-moment map (sign +
    magnitude), ``signed=False`` the second-moment (sqrt-spaced, non-negative)
    map; ``bits`` 4 packs two codes per byte.  ``bits=32`` keeps fp32."""

    def __init__(self, like: torch.Tensor, bits: int, signed: bool):
        self.shape, self.n = like.shape, like.numel()
        self.bits, self.signed = bits, signed
        dev = like.device
        if bits == 32:
            self.full = torch.zeros(self.n, dtype=torch.float32, device=dev)
            return
        npad = _pad(self.n)
        self.codes = torch.zeros(npad // 2 if bits == 4 else npad, dtype=torch.uint8, device=dev)
        self.scale = torch.zeros(npad // GROUP, dtype=torch.float32, device=dev)

    def decode(self) -> torch.Tensor:
        if self.bits == 32:
            return self.full.clone().view(self.shape)
        G = self.scale.numel()
        c = _unpack4(self.codes) if self.bits == 4 else self.codes
        x = (dequant_m if self.signed else dequant_v)(c.view(G, GROUP), self.scale, self.bits)
        x = torch.where(self.scale[:, None] > 0, x, torch.zeros_like(x))
        return x.view(-1)[:self.n].view(self.shape)

    def encode(self, x: torch.Tensor):
        if self.bits == 32:
            self.full.copy_(x.reshape(-1))
            return
        G = self.scale.numel()
        buf = torch.zeros(G * GROUP, dtype=torch.float32, device=x.device)
        buf[:self.n] = x.reshape(-1).float()
        codes, scale = (quant_m if self.signed else quant_v)(buf.view(G, GROUP), self.bits)
        self.codes.copy_(_pack4(codes.view(-1)) if self.bits == 4 else codes.view(-1))
        self.scale.copy_(scale)

    def nbytes(self) -> int:
        if self.bits == 32:
            return self.full.numel() * 4
        return self.codes.numel() + self.scale.numel() * 4


def _rms(t: torch.Tensor) -> torch.Tensor:
    return t.norm(2) / (t.numel() ** 0.5)


def _approx_sq(row: torch.Tensor, col: torch.Tensor) -> torch.Tensor:
    r = (row / row.mean(dim=-1, keepdim=True)).rsqrt_().unsqueeze(-1)
    c = col.unsqueeze(-2).rsqrt()
    return r * c


class _LowBitBase(torch.optim.Optimizer):
    def __init__(self, params, defaults, q_bits: int, threshold: int):
        if q_bits not in (4, 8, 32):
            raise ValueError("q_bits must be 4, 8 or 32")
        defaults = dict(defaults, q_bits=q_bits, threshold=threshold)
        super().__init__(params, defaults)

    def _q(self, p, group, signed: bool) -> QState:
        bits = group["q_bits"] if p.numel() >= group["threshold"] else 32
        return QState(p, bits, signed)

    def state_bytes(self) -> int:
        total = 0
        for st in self.state.values():
            for v in st.values():
                if isinstance(v, QState):
                    total += v.nbytes()
                elif torch.is_tensor(v):
                    total += v.numel() * v.element_size()
        return total


class Q_AGD(_LowBitBase):  # noqa: N801 (reference name)
    """AGD (``optimizers/agd.py``) with 4/8-bit first and second moments.
    Parity: ``atorch/optimizers/low_bit/optim/q_agd.py``."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), delta=1e-5, weight_decay=0.0, amsgrad=False,
                 clip=None, q_bits: int = 4, threshold: int = 4096):
        super().__init__(params, dict(lr=lr, betas=betas, delta=delta, weight_decay=weight_decay,
                                      amsgrad=amsgrad, clip=clip), q_bits, threshold)

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
                g = p.grad.float()
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = self._q(p, grp, True)
                    st["exp_avg_sq"] = self._q(p, grp, False)
                    if grp["amsgrad"]:
                        st["max_exp_avg_sq"] = self._q(p, grp, False)
                st["step"] += 1
                t = st["step"]
                m, v = st["exp_avg"].decode(), st["exp_avg_sq"].decode()
                bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
                prev = m / (1 - b1 ** (t - 1)) if t > 1 else torch.zeros_like(m)
                m.mul_(b1).add_(g, alpha=1 - b1)
                diff = m / bc1 - prev
                v.mul_(b2).addcmul_(diff, diff, value=1 - b2)
                if grp["amsgrad"]:
                    vmax = torch.maximum(st["max_exp_avg_sq"].decode(), v)
                    st["max_exp_avg_sq"].encode(vmax)
                    den = vmax.sqrt()
                else:
                    den = v.sqrt()
                den.clamp_(min=grp["delta"] * math.sqrt(bc2))
                upd = m / den
                if grp["clip"] is not None:
                    upd.clamp_(-grp["clip"], grp["clip"])
                pf = p.float()
                if wd:
                    pf.mul_(1.0 - lr * wd)
                pf.add_(upd, alpha=-lr * math.sqrt(bc2) / bc1)
                p.copy_(pf)
                st["exp_avg"].encode(m)
                st["exp_avg_sq"].encode(v)
        return loss


class Q_Adafactor(_LowBitBase):  # noqa: N801 (reference name)
    """Adafactor with factored second moments for >= 2-D parameters (row /
    column statistics stay fp32: they are tiny) and quantized first moment /
    unfactored second moment.  Parity:
    ``atorch/optimizers/low_bit/optim/q_adafactor.py`` (same hyper-parameters:
    relative_step, scale_parameter, warmup_init, decay_rate, clip_threshold)."""

    def __init__(self, params, lr=None, eps2=(1e-30, 1e-3), clip_threshold=1.0, decay_rate=-0.8, beta1=None,
                 weight_decay=0.0, scale_parameter=True, relative_step=True, warmup_init=False, q_bits: int = 4,
                 threshold: int = 4096):
        if lr is not None and relative_step:
            relative_step = False  # an explicit lr wins
        if lr is None and not relative_step:
            raise ValueError("lr is required when relative_step=False")
        super().__init__(params, dict(lr=lr, eps2=eps2, clip_threshold=clip_threshold, decay_rate=decay_rate,
                                      beta1=beta1, weight_decay=weight_decay, scale_parameter=scale_parameter,
                                      relative_step=relative_step, warmup_init=warmup_init), q_bits, threshold)

    @staticmethod
    def _lr(grp, st):
        rel = grp["lr"]
        if grp["relative_step"]:
            min_step = 1e-6 * st["step"] if grp["warmup_init"] else 1e-2
            rel = min(min_step, 1.0 / math.sqrt(st["step"]))
        scale = max(grp["eps2"][1], float(st["RMS"])) if grp["scale_parameter"] else 1.0
        return scale * rel

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for grp in self.param_groups:
            for p in grp["params"]:
                if p.grad is None:
                    continue
                g = p.grad.float()
                st = self.state[p]
                factored = g.dim() >= 2
                if not st:
                    st["step"] = 0
                    if grp["beta1"] is not None:
                        st["exp_avg"] = self._q(p, grp, True)
                    if factored:
                        st["exp_avg_sq_row"] = torch.zeros(g.shape[:-1], device=p.device)
                        st["exp_avg_sq_col"] = torch.zeros(g.shape[:-2] + g.shape[-1:], device=p.device)
                    else:
                        st["exp_avg_sq"] = self._q(p, grp, False)
                st["step"] += 1
                pf = p.float()
                st["RMS"] = _rms(pf)
                lr = self._lr(grp, st)
                beta2t = 1.0 - math.pow(st["step"], grp["decay_rate"])
                upd = g * g + grp["eps2"][0]
                if factored:
                    row, col = st["exp_avg_sq_row"], st["exp_avg_sq_col"]
                    row.mul_(beta2t).add_(upd.mean(dim=-1), alpha=1.0 - beta2t)
                    col.mul_(beta2t).add_(upd.mean(dim=-2), alpha=1.0 - beta2t)
                    upd = _approx_sq(row, col).mul_(g)
                else:
                    v = st["exp_avg_sq"].decode()
                    v.mul_(beta2t).add_(upd, alpha=1.0 - beta2t)
                    st["exp_avg_sq"].encode(v)
                    upd = v.rsqrt().mul_(g)
                upd.div_(max(1.0, float(_rms(upd)) / grp["clip_threshold"]))
                upd.mul_(lr)
                if grp["beta1"] is not None:
                    m = st["exp_avg"].decode()
                    m.mul_(grp["beta1"]).add_(upd, alpha=1 - grp["beta1"])
                    st["exp_avg"].encode(m)
                    upd = m
                if grp["weight_decay"]:
                    pf.mul_(1 - grp["weight_decay"] * lr)
                pf.sub_(upd)
                p.copy_(pf)
        return loss


class Q_CAME(_LowBitBase):  # noqa: N801 (reference name)
    """CAME (confidence-guided adaptive memory-efficient optimisation):
    Adafactor-style factored second moment plus a factored "instability"
    statistic of (update - exp_avg)^2 that scales the first moment.  Parity:
    ``atorch/optimizers/low_bit/optim/q_came.py``."""

    def __init__(self, params, lr=None, eps=(1e-30, 1e-16), clip_threshold=1.0, betas=(0.9, 0.999, 0.9999),
                 weight_decay=0.0, q_bits: int = 4, threshold: int = 4096):
        if lr is None:
            raise ValueError("Q_CAME needs an explicit lr")
        super().__init__(params, dict(lr=lr, eps=eps, clip_threshold=clip_threshold, betas=betas,
                                      weight_decay=weight_decay), q_bits, threshold)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for grp in self.param_groups:
            b1, b2, b3 = grp["betas"]
            for p in grp["params"]:
                if p.grad is None:
                    continue
                g = p.grad.float()
                st = self.state[p]
                factored = g.dim() >= 2
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = self._q(p, grp, True)
                    if factored:
                        for k, shp in (("exp_avg_sq_row", g.shape[:-1]), ("exp_avg_sq_col", g.shape[:-2] + g.shape[-1:]),
                                       ("exp_avg_res_row", g.shape[:-1]),
                                       ("exp_avg_res_col", g.shape[:-2] + g.shape[-1:])):
                            st[k] = torch.zeros(shp, device=p.device)
                    else:
                        st["exp_avg_sq"] = self._q(p, grp, False)
                st["step"] += 1
                upd = g * g + grp["eps"][0]
                if factored:
                    st["exp_avg_sq_row"].mul_(b2).add_(upd.mean(dim=-1), alpha=1.0 - b2)
                    st["exp_avg_sq_col"].mul_(b2).add_(upd.mean(dim=-2), alpha=1.0 - b2)
                    upd = _approx_sq(st["exp_avg_sq_row"], st["exp_avg_sq_col"]).mul_(g)
                else:
                    v = st["exp_avg_sq"].decode()
                    v.mul_(b2).add_(upd, alpha=1.0 - b2)
                    st["exp_avg_sq"].encode(v)
                    upd = v.rsqrt().mul_(g)
                upd.div_((_rms(upd) / grp["clip_threshold"]).clamp_(min=1.0))
                m = st["exp_avg"].decode()
                m.mul_(b1).add_(upd, alpha=1 - b1)
                st["exp_avg"].encode(m)
                if factored:
                    res = (upd - m) ** 2 + grp["eps"][1]
                    st["exp_avg_res_row"].mul_(b3).add_(res.mean(dim=-1), alpha=1.0 - b3)
                    st["exp_avg_res_col"].mul_(b3).add_(res.mean(dim=-2), alpha=1.0 - b3)
                    upd = _approx_sq(st["exp_avg_res_row"], st["exp_avg_res_col"]).mul_(m)
                else:
                    upd = m
                pf = p.float()
                if grp["weight_decay"]:
                    pf.mul_(1 - grp["weight_decay"] * grp["lr"])
                pf.add_(upd, alpha=-grp["lr"])
                p.copy_(pf)
        return loss
