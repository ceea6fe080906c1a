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

Parity: ATorch ``atorch/optimizers/low_bit/optim/q_adamw.py`` (``Q_AdamW``,
``q_bits``, ``threshold``; ATorch also ships Q_AGD / Q_CAME / Q_Adafactor on
the same quantizer -- ``Q_AGD`` here reuses the AGD math with quantized
states through the reference path).
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
