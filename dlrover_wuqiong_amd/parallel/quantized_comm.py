"""Quantized collectives (ZeRO++ qwZ / qgZ) over RCCL.

* ``quantized_all_gather`` (qwZ): each rank quantizes its shard to int8
  (or int4) + per-group {1/scale, zero point}; ONE all-gather moves the
  codes and ONE the params; the receiver dequantizes the whole gathered
  tensor in one kernel.  Wire bytes per element: 1 (0.5) instead of 2 (bf16).
* ``quantized_reduce_scatter`` (qgZ): each rank quantizes its full gradient
  (N destination slices, groups never straddle a slice); ONE all-to-all
  delivers slice r of every rank to rank r; ``dequant_reduce`` sums the N
  quantized slices in fp32 registers and writes the reduced shard once.
  Within an MI355X node the 8 GPUs are fully connected by xGMI, so the
  all-to-all is a single hop on every link -- no hierarchical swizzle
  (the reference's multi-node ``swizzle_quant`` layout) is needed.
* ``quantized_all_reduce`` = qgZ reduce-scatter + qwZ all-gather of the
  reduced shard (averaging optional).

Error: per-group relative error ~ 1 / 2^(bits-1) of the group's absmax;
the reduce step dequantizes in fp32 before summing, so error does not
compound with N.

Parity: ATorch quantizer ops ``swizzle_quant`` / ``quantized_reduction``
(``atorch/ops/csrc/quantization/{swizzled_quantize,quant_reduce}.cu``,
``pt_binding.cpp:157-177``) and ``CUDAQuantizer``.
"""

from typing import Optional

import torch
import torch.distributed as dist

from ..ops.quantization import dequant_reduce, quantize


def _ws(group) -> int:
    return dist.get_world_size(group)


def _gs_for(elems: int, group_size: int) -> int:
    gs = min(group_size, elems)
    gs -= gs % 8
    while gs > 8 and elems % gs:
        gs -= 8
    if gs <= 0 or elems % gs:
        raise ValueError(f"no group size (multiple of 8) divides {elems}")
    return gs


def quantized_all_gather(x: torch.Tensor, group=None, bits: int = 8, group_size: int = 2048,
                         out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """Every rank's ``x`` ([n], n % 8 == 0, same n everywhere) -> [N * n]
    in rank order, dequantized to ``out_dtype`` (default x.dtype)."""
    n_ranks = _ws(group)
    x = x.reshape(-1)
    n = x.numel()
    gs = _gs_for(n, group_size)
    codes, params = quantize(x, n // gs, bits, symmetric=True)
    all_codes = torch.empty(n_ranks * codes.numel(), dtype=torch.int8, device=x.device)
    all_params = torch.empty(n_ranks * params.numel(), dtype=torch.float32, device=x.device)
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(all_codes.view(n_ranks, -1).unbind(0)), codes, group=group)
        dist.all_gather(list(all_params.view(n_ranks, -1).unbind(0)), params.reshape(-1), group=group)
    else:
        dist.all_gather_into_tensor(all_codes, codes, group=group)
        dist.all_gather_into_tensor(all_params, params.reshape(-1), group=group)
    dt = out_dtype or x.dtype
    # one dequantize over the concatenation: N * n elements, same group size
    return dequant_reduce(all_codes, all_params, 1, n_ranks * n, gs, bits,
                          dtype=dt if dt in (torch.float32, torch.bfloat16) else torch.float32).to(dt)


def quantized_reduce_scatter(x: torch.Tensor, group=None, bits: int = 8, group_size: int = 2048,
                             out_dtype: Optional[torch.dtype] = None, average: bool = False) -> torch.Tensor:
    """Sum over ranks of ``x`` ([N * m]) -> this rank's slice [m]."""
    n_ranks = _ws(group)
    x = x.reshape(-1)
    if x.numel() % n_ranks:
        raise ValueError("tensor size must divide by the group size")
    m = x.numel() // n_ranks
    gs = _gs_for(m, group_size)
    codes, params = quantize(x, x.numel() // gs, bits, symmetric=True)
    recv_c = torch.empty_like(codes)
    recv_p = torch.empty_like(params)
    dist.all_to_all_single(recv_c, codes, group=group)
    dist.all_to_all_single(recv_p, params, group=group)
    dt = out_dtype or x.dtype
    out = dequant_reduce(recv_c, recv_p, n_ranks, m, gs, bits,
                         dtype=dt if dt in (torch.float32, torch.bfloat16) else torch.float32)
    if average:
        out.div_(n_ranks)
    return out.to(dt)


def quantized_all_reduce(x: torch.Tensor, group=None, bits: int = 8, group_size: int = 2048,
                         average: bool = False) -> torch.Tensor:
    """In place: x <- sum (or mean) over ranks, through a quantized
    reduce-scatter and a quantized all-gather of the reduced shard."""
    n_ranks = _ws(group)
    flat = x.reshape(-1)
    n = flat.numel()
    pad = (-n) % (8 * n_ranks)
    src = torch.cat([flat, flat.new_zeros(pad)]) if pad else flat
    shard = quantized_reduce_scatter(src, group, bits, group_size, out_dtype=torch.float32, average=average)
    full = quantized_all_gather(shard, group, bits, group_size, out_dtype=torch.float32)
    x.copy_(full[:n].view_as(x))
    return x
