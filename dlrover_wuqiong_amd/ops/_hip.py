"""Glue between PyTorch tensors and the HIP kernel library.

Tensors on a GPU always run the hand-written gfx950 kernels; if the kernel
library cannot be loaded on a GPU host this raises (no silent eager
fallback).  CPU tensors run the PyTorch reference math - that is the CPU/gloo
execution path of the framework, also used as the numerics oracle in tests.
"""

import ctypes

import torch

from .._native import kernels


class HipKernelError(RuntimeError):
    pass


_TIMER = None  # utils.xpu_timer.XpuTimer timing this framework's own kernels (install(kernels=True))
_NO_LAUNCH = ("workspace", "error", "_size", "mem_get_info", "ipc_", "device_malloc", "device_free",
              "event_sync", "stream_sync", "_xt_", "det_floats")


class _TimedLib:
    """The kernel library with every launching ``dw_*`` entry point bracketed
    by xpu_timer events on torch's current stream (the stream every launcher
    of ``ops/*`` passes), so the framework's own HIP kernels -- attention,
    norms, fused Adam, hipBLASLt epilogue GEMMs -- show up next to the
    torch-level GEMMs and collectives (the reference gets this from an
    LD_PRELOAD hook of the vendor libraries: atorch/dev/xpu_timer)."""

    def __init__(self, lib_, timer):
        self._lib, self._timer = lib_, timer

    def __getattr__(self, name):
        f = getattr(self._lib, name)
        if not name.startswith("dw_") or any(t in name for t in _NO_LAUNCH):
            return f
        timer = self._timer

        def call(*args):
            with timer.kernel(name):
                return f(*args)

        return call


def lib():
    L = kernels(required=True)
    return _TimedLib(L, _TIMER) if _TIMER is not None else L


def stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t) -> ctypes.c_void_p:
    if t is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(t.data_ptr())


def check(err: int, what: str = "kernel"):
    if err != 0:
        msg = lib().dw_hip_error_string(err)
        raise HipKernelError(f"{what} failed: hip error {err} ({msg.decode() if msg else '?'})")


def use_hip(t: torch.Tensor) -> bool:
    return t.is_cuda


def bf16_path(t: torch.Tensor) -> bool:
    """Whether a bf16-only kernel takes ``t``: a bf16 GPU tensor, or an fp32
    one inside a bf16 autocast region (``amp_native`` over fp32 weights).
    fp32 outside autocast runs the fp32 PyTorch math instead of silently
    dropping to bf16."""
    if not use_hip(t):
        return False
    if t.dtype == torch.bfloat16:
        return True
    return (t.dtype == torch.float32 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16)


def bf16(*ts):
    """Operands of a bf16 kernel: floating tensors cast to bf16 (autograd
    tracks the cast, so fp32 parameters get fp32 gradients)."""
    out = tuple(t.to(torch.bfloat16) if (t is not None and t.is_floating_point() and t.dtype != torch.bfloat16)
                else t for t in ts)
    return out if len(out) != 1 else out[0]


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    raise HipKernelError(f"unsupported dtype {t.dtype} for HIP kernel")


def require_bf16(*ts):
    for t in ts:
        if t is not None and t.dtype != torch.bfloat16:
            raise HipKernelError(f"HIP kernel expects bf16 tensors, got {t.dtype}")


_ZERO_WS = {}
_GRID_WS = {}


def grid_sum_ws(device) -> torch.Tensor:
    """Scratch of the deterministic grid sums (dw_common.h grid_sum_finish):
    2048 partials (any content) + a counter word that is zero between calls.
    Its own buffer per (device, stream) -- not the zeroed workspace, whose
    every word must stay zero."""
    key = (torch.device(device).index, torch.cuda.current_stream(device).cuda_stream)
    buf = _GRID_WS.get(key)
    if buf is None:
        buf = _GRID_WS[key] = torch.zeros(2048 + 1, device=device, dtype=torch.float32)
    return buf


_DET_WS = {}


def deterministic() -> bool:
    """Bit-reproducible gradients: ``DWAMD_DETERMINISTIC=1`` or
    ``torch.use_deterministic_algorithms(True)``.  The column-reduction
    kernels (bias / norm-weight gradients) then combine per-block partials in
    a fixed order instead of with float atomics (csrc/kernels/colred.hip)."""
    import os

    return os.environ.get("DWAMD_DETERMINISTIC", "0") == "1" or torch.are_deterministic_algorithms_enabled()


def det_scratch(rows: int, C: int, kind: int, device):
    """Pointer to the fp32 partial-sum scratch of a deterministic column
    reduction (``kind``: 0 colsum, 1 GELU-bias backward, 2 norm backward),
    or a null pointer when deterministic mode is off.  Any content; one
    buffer per (device, stream), grown on demand."""
    if not deterministic():
        return ctypes.c_void_p(0)
    n = int(kernels(required=True).dw_colred_det_floats(int(rows), int(C), int(kind)))
    key = (torch.device(device).index, torch.cuda.current_stream(device).cuda_stream)
    buf = _DET_WS.get(key)
    if buf is None or buf.numel() < n:
        buf = _DET_WS[key] = torch.empty(max(n, 1 << 16), device=device, dtype=torch.float32)
    return ptr(buf)


def zeroed_workspace(nfloats: int, device) -> torch.Tensor:
    """fp32 scratch that is all-zero on entry to a kernel and left all-zero by
    it (the column-reduction kernels clear what they consume).  One buffer per
    (device, stream): stream order serializes its users, and no per-call
    memset launch is needed."""
    key = (torch.device(device).index, torch.cuda.current_stream(device).cuda_stream)
    buf = _ZERO_WS.get(key)
    if buf is None or buf.numel() < nfloats:
        buf = torch.zeros(max(nfloats, 1 << 16), device=device, dtype=torch.float32)
        _ZERO_WS[key] = buf
    return buf
