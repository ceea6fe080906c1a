"""Grouped (per-expert) linear layers on one HIP launch per GEMM
(``csrc/kernels/grouped_gemm.hip``).

``grouped_linear(x, w, offs)``: rows ``[offs[e], offs[e+1])`` of ``x`` [T, K]
go through expert ``e``'s weight ``w[e]`` [N, K] (nn.Linear layout) ->
[T, N].  ``offs`` ([E+1] int32) stays on the device, so an MoE layer never
synchronises with the host to read its per-expert token counts.  Backward:
dX by the NN form, dW by the TN form (one launch each, reduction over each
group's rows).

CPU tensors run the per-expert PyTorch loop (reference math / gloo path).

Parity: ATorch grouped-GEMM experts (atorch/atorch/modules/moe/
grouped_gemm_moe.py:46-112).
"""

from typing import List, Union

import torch
import torch.nn.functional as F

from . import _hip

MODE_NT, MODE_NN, MODE_TN = 0, 1, 2


def offsets_from_counts(counts: Union[torch.Tensor, List[int]], device) -> torch.Tensor:
    """[E] counts (device tensor or host list) -> [E+1] int32 offsets on ``device``."""
    if not torch.is_tensor(counts):
        counts = torch.tensor(list(counts), dtype=torch.int64)
    c = counts.to(device=device, dtype=torch.int64, non_blocking=True)
    offs = torch.zeros(c.numel() + 1, dtype=torch.int32, device=device)
    torch.cumsum(c, 0, out=offs[1:])
    return offs


def _launch(mode, A, B, C, offs, E, T, M, Nout, R, lda, ldb, ldc, b_es, c_es):
    _hip.check(_hip.lib().dw_grouped_gemm(mode, _hip.ptr(A), _hip.ptr(B), _hip.ptr(C), _hip.ptr(offs), E, T, M, Nout,
                                          R, lda, ldb, ldc, b_es, c_es, _hip.stream()), "grouped_gemm")


def _check_shapes(x, w):
    T, K = x.shape
    E, N, K2 = w.shape
    if K2 != K:
        raise ValueError(f"grouped_linear: x [{T}, {K}] vs w [{E}, {N}, {K2}]")
    if K % 8 or N % 8:
        raise _hip.HipKernelError(f"grouped GEMM needs K and N divisible by 8 (got K={K}, N={N})")
    return T, K, E, N


class _GroupedLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, offs):
        _hip.require_bf16(x, w)
        x, w = x.contiguous(), w.contiguous()
        T, K, E, N = _check_shapes(x, w)
        y = torch.empty(T, N, device=x.device, dtype=x.dtype)
        if T > 0:
            _launch(MODE_NT, x, w, y, offs, E, T, 0, N, K, K, K, N, N * K, 0)
        ctx.save_for_backward(x, w, offs)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, offs = ctx.saved_tensors
        dy = dy.contiguous().to(torch.bfloat16)
        T, K = x.shape
        E, N, _ = w.shape
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            if T > 0:
                _launch(MODE_NN, dy, w, dx, offs, E, T, 0, K, N, N, K, K, N * K, 0)
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w)
            _launch(MODE_TN, dy, x, dw, offs, E, T, N, K, 0, N, K, K, 0, N * K)
        return dx, dw, None


def grouped_linear_reference(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """Per-expert loop (autograd-able): the CPU path and the numerics oracle."""
    o = offs.tolist()
    outs = [F.linear(x[o[e]:o[e + 1]], w[e]) for e in range(w.shape[0])]
    y = torch.cat(outs, 0) if outs else x.new_zeros((0, w.shape[1]))
    if y.shape[0] == 0:
        y = y + 0 * w.sum()  # keep w in the graph
    return y


def grouped_linear(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """x [T, K] (rows grouped by expert), w [E, N, K], offs [E+1] int32 -> [T, N]."""
    if _hip.use_hip(x):
        return _GroupedLinearFn.apply(x, w, offs.to(device=x.device, dtype=torch.int32))
    return grouped_linear_reference(x, w, offs)
