"""Group-wise int8 / int4 quantization (HIP kernels ``quant.hip``).

``quantize(x, groups, bits, symmetric) -> (codes int8, params fp32 [groups, 2])``
and ``dequantize(codes, params, groups, bits, symmetric, dtype)`` follow the
ATorch / DeepSpeed quantizer format (params = {1/scale, zero point}; int4
packs two codes per byte, first in the high nibble), so quantized tensors
are interchangeable.  ``Quantizer`` is the ``CUDAQuantizer`` interface
(adaptive group count: groups of <= 8k elements dividing the tensor).

Parity: ATorch ``atorch/ops/quantizer/__init__.py`` (CUDAQuantizer),
``atorch/ops/csrc/quantization/{quantize,dequantize,quant_reduce}.cu`` and
``atorch/tests/common_tests/test_quantize.py`` (the fp32 reference math
below is that test's formula).
"""

import math
from typing import Optional, Tuple

import torch

from . import _hip


def _q_props(bits: int):
    return float(2 ** bits), float(-(2 ** (bits - 1))), float(2 ** (bits - 1) - 1)


def quantize_reference(x: torch.Tensor, groups: int, bits: int = 8, symmetric: bool = True):
    qrange, qmin, qmax = _q_props(bits)
    xf = x.reshape(groups, -1).float()
    if symmetric:
        amax = xf.abs().amax(-1, keepdim=True)
        scale = torch.where(amax == 0, torch.ones_like(amax), qrange / (2 * amax))
        zp = torch.zeros_like(scale)
        v = xf * scale
    else:
        mx, mn = xf.amax(-1, keepdim=True), xf.amin(-1, keepdim=True)
        scale = torch.where(mx == mn, torch.ones_like(mx), qrange / (mx - mn))
        zp = qmin - mn * scale
        v = xf * scale + zp
    c = torch.round(v).clamp(qmin, qmax).to(torch.int8)
    params = torch.cat([1.0 / scale, zp], dim=-1)
    if bits == 4:
        c = c.view(-1, 2)
        c = ((c[:, 0].to(torch.int32) & 0xF) << 4 | (c[:, 1].to(torch.int32) & 0xF)).to(torch.uint8).view(torch.int8)
    return c.reshape(-1), params


def _unpack4(c: torch.Tensor) -> torch.Tensor:
    b = c.to(torch.int32)
    hi = b >> 4
    lo = ((b & 0xF) ^ 0x8) - 0x8
    return torch.stack([hi, lo], dim=-1).reshape(-1)


def dequantize_reference(c: torch.Tensor, params: torch.Tensor, groups: int, bits: int = 8,
                         dtype=torch.float32) -> torch.Tensor:
    codes = _unpack4(c) if bits == 4 else c.to(torch.int32)
    f = codes.float().reshape(groups, -1)
    return ((f - params[:, 1:2]) * params[:, 0:1]).reshape(-1).to(dtype)


def _check(x: torch.Tensor, groups: int, bits: int):
    if bits not in (4, 8):
        raise ValueError("bits must be 8 or 4")
    n = x.numel()
    if groups <= 0 or n % groups or (n // groups) % 8:
        raise ValueError(f"{n} elements do not split into {groups} groups of a multiple of 8")


def quantize(x: torch.Tensor, groups: int, bits: int = 8, symmetric: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """x (fp32 / bf16, any shape) -> (codes int8 [n or n/2], params fp32 [groups, 2])."""
    _check(x, groups, bits)
    if not _hip.use_hip(x):
        return quantize_reference(x, groups, bits, symmetric)
    x = x.contiguous()
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    if x.data_ptr() % 16:
        x = x.clone()
    n = x.numel()
    q = torch.empty(n if bits == 8 else n // 2, dtype=torch.int8, device=x.device)
    params = torch.empty(groups, 2, dtype=torch.float32, device=x.device)
    _hip.check(_hip.lib().dw_quantize(_hip.ptr(x), _hip.dtype_code(x), _hip.ptr(q), _hip.ptr(params), groups,
                                      n // groups, bits, int(symmetric), _hip.stream()), "quantize")
    return q, params


def dequant_reduce(codes: torch.Tensor, params: torch.Tensor, n_src: int, elems: int, group_size: int,
                   bits: int = 8, out: Optional[torch.Tensor] = None, dtype=torch.float32,
                   accumulate: bool = False) -> torch.Tensor:
    """Sum of ``n_src`` quantized chunks (codes [n_src, elems(/2)], params
    [n_src, elems / group_size, 2]) -> [elems] (the receive side of a
    quantized reduce-scatter; ``n_src = 1`` is a plain dequantize)."""
    if out is None:
        out = (torch.zeros if accumulate else torch.empty)(elems, dtype=dtype, device=codes.device)
    if not _hip.use_hip(codes):
        gpc = elems // group_size
        cs = codes.reshape(n_src, -1)
        ps = params.reshape(n_src, gpc, 2)
        tot = sum(dequantize_reference(cs[i], ps[i], gpc, bits) for i in range(n_src))
        if accumulate:
            out += tot.to(out.dtype)
        else:
            out.copy_(tot.view_as(out))
        return out
    assert out.is_contiguous() and out.numel() == elems and out.data_ptr() % 16 == 0
    _hip.check(_hip.lib().dw_dequant_reduce(_hip.ptr(codes.contiguous()), _hip.ptr(params.contiguous()),
                                            _hip.ptr(out), _hip.dtype_code(out), int(n_src), int(elems),
                                            int(group_size), bits, int(accumulate), _hip.stream()),
               "dequant_reduce")
    return out


def dequantize(codes: torch.Tensor, params: torch.Tensor, groups: int, bits: int = 8, symmetric: bool = True,
               dtype=torch.float32) -> torch.Tensor:
    n = codes.numel() * (2 if bits == 4 else 1)
    return dequant_reduce(codes, params, 1, n, n // groups, bits, dtype=dtype)


def choose_groups(numel: int, target_group_size: int = 8000, max_group_size: int = 16000) -> int:
    """Adaptive group count: groups of a multiple of 8 elements dividing
    ``numel``, close to ``target_group_size`` (CUDAQuantizer's rule)."""
    if numel % 8:
        raise ValueError(f"quantized tensors need a multiple of 8 elements, got {numel}")
    groups = max(1, math.ceil(numel / target_group_size))
    while groups < numel and numel % (8 * groups):
        groups += 1
    while numel % (16 * groups) == 0 and numel / groups > target_group_size:
        groups *= 2
    if numel / groups >= max_group_size:
        raise ValueError(f"no group size under {max_group_size} divides {numel}")
    return groups


class Quantizer:
    """``CUDAQuantizer`` interface: ``quantize(param, groups=None) -> (codes,
    params)`` (symmetric int8, adaptive groups) and ``dequantize(codes,
    params) -> fp``.  ``bits=4`` halves the bytes again."""

    target_group_size = 8000

    def __init__(self, bits: int = 8, symmetric: bool = True):
        self.bits, self.symmetric = bits, symmetric
        self._groups = {}

    def groups_for(self, numel: int) -> int:
        g = self._groups.get(numel)
        if g is None:
            g = self._groups[numel] = choose_groups(numel, self.target_group_size)
        return g

    def quantize(self, param: torch.Tensor, groups: Optional[int] = None):
        groups = groups or self.groups_for(param.numel())
        return quantize(param, groups, self.bits, self.symmetric)

    def dequantize(self, codes: torch.Tensor, params: torch.Tensor, dtype=torch.float32):
        return dequantize(codes, params, params.shape[0], self.bits, self.symmetric, dtype)
