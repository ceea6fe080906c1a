"""FP8 linear layers with delayed scaling on the CDNA4 FP8 matrix cores.

MI355X's MFMA consumes OCP e4m3 / e5m2 at twice the bf16 rate.  An
``Fp8Linear`` runs its three GEMMs in FP8 (hipBLASLt kernels through
``torch._scaled_mm``):

    forward   y  = x8 @ w8^T            x8, w8: e4m3
    backward  dx = g8 @ w8              g8: e5m2 ("HYBRID") or e4m3 ("E4M3")
              dw = g8^T @ x8

Every FP8 operand comes from ``dw_fp8_cast_amax`` (``csrc/kernels/fp8.hip``):
one pass that scales by the tensor's current factor, saturates, converts 8
values per lane with the gfx950 ``v_cvt_pk_fp8/bf8_f32`` instructions and
records this pass's amax.  The factors follow Transformer Engine's delayed
scaling: after each optimizer step ONE kernel (``Fp8State.update``) pushes
every tensor's recorded amax into its history and sets ``scale = fmax /
(max(history) * 2^margin)`` for the next step -- no host sync anywhere.
``reduce_amax`` takes the MAX of the recorded amaxes over the data-parallel
group first (one all-reduce per step), so every rank quantises alike.

CPU tensors run the same math with torch's float8 dtypes (the numerics
oracle of the tests).

Parity: ATorch ``auto/opt_lib/amp_optimization.py`` ``Fp8Optimization``
(Transformer Engine ``te.Linear`` + ``fp8_autocast(DelayedScaling)``);
include / exclude / margin / interval / fp8_format / amax_history_len /
amax_compute_algo / reduce_amax keep their meaning.
"""

import math
from typing import Dict, Iterable, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _hip

FP8_MAX = {"e4m3": 448.0, "e5m2": 57344.0}
_TORCH_DT = {"e4m3": torch.float8_e4m3fn, "e5m2": torch.float8_e5m2}


class Fp8State:
    """Delayed-scaling metadata of every FP8 tensor role on one device, in
    contiguous buffers so one kernel updates all of them."""

    def __init__(self, device, history_len: int = 1024, margin: int = 0, algo: str = "max",
                 capacity: int = 8192, group=None, reduce_amax: bool = True, interval: int = 1):
        self.device = torch.device(device)
        self.h = history_len if algo == "max" else 1
        self.margin = margin
        self.cap = capacity
        self.group = group
        self.reduce_amax = reduce_amax
        self.interval = max(1, int(interval))
        d = self.device
        self.amax_bits = torch.zeros(capacity, dtype=torch.int32, device=d)  # float bits, this step
        self.hist = torch.zeros(capacity, self.h, dtype=torch.float32, device=d)
        self.fmax = torch.ones(capacity, dtype=torch.float32, device=d)
        self.scale = torch.ones(capacity, dtype=torch.float32, device=d)
        self.inv_scale = torch.ones(capacity, dtype=torch.float32, device=d)
        self.n = 0
        self.steps = 0
        self.head = 0  # ring slot of the history the next update writes

    def register(self, fmt: str) -> int:
        if self.n >= self.cap:
            raise RuntimeError(f"Fp8State: more than {self.cap} FP8 tensors")
        i = self.n
        self.n += 1
        self.fmax[i] = FP8_MAX[fmt]
        return i

    @torch.no_grad()
    def update(self):
        """Amax of the finished step -> history -> next scales (every
        ``interval`` steps; call after ``optimizer.step()``)."""
        self.steps += 1
        if self.n == 0 or self.steps % self.interval:
            return
        amax = self.amax_bits[: self.n]
        if self.reduce_amax and self.group is not False:
            import torch.distributed as dist

            if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
                # non-negative float bits order like the floats: MAX on int32
                dist.all_reduce(amax, op=dist.ReduceOp.MAX, group=self.group)
        mp = float(2.0 ** self.margin)
        head = self.head
        self.head = (self.head + 1) % self.h  # the history is a ring: no shifting
        if _hip.use_hip(self.amax_bits):
            _hip.check(_hip.lib().dw_fp8_update_scales(
                _hip.ptr(self.amax_bits), _hip.ptr(self.hist), _hip.ptr(self.fmax), _hip.ptr(self.scale),
                _hip.ptr(self.inv_scale), self.n, self.h, head, mp, _hip.stream()), "fp8_update_scales")
            return
        n = self.n
        cur = amax.view(torch.float32).clone()
        self.hist[:n, head] = cur
        best = self.hist[:n].amax(1)
        ok = (best > 0) & torch.isfinite(best)
        sc = torch.where(ok, self.fmax[:n] / (best * mp), self.scale[:n])
        sc = torch.where(torch.isinf(best), self.scale[:n] * 0.5, sc)
        self.scale[:n] = sc
        self.inv_scale[:n] = 1.0 / sc
        amax.zero_()


_STATES: Dict[torch.device, Fp8State] = {}
_DEFAULTS: dict = {}


def fp8_state(device, **kw) -> Fp8State:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    st = _STATES.get(d)
    if st is None:
        st = _STATES[d] = Fp8State(d, **dict(_DEFAULTS, **kw))
    return st


def configure(**kw):
    """Defaults (history_len, margin, algo, group, reduce_amax, interval) for
    states created after this call."""
    _DEFAULTS.update(kw)


def fp8_update():
    """Advance every device's delayed scaling (after ``optimizer.step()``)."""
    for st in _STATES.values():
        st.update()


@torch.no_grad()
def cast_to_fp8(x: torch.Tensor, st: Fp8State, idx: int, fmt: str) -> torch.Tensor:
    """x (bf16 / fp32) -> float8 tensor scaled by ``st.scale[idx]``; records
    amax(|x|) of this call into ``st.amax_bits[idx]``."""
    x = x.contiguous()
    if _hip.use_hip(x) and x.dtype in (torch.bfloat16, torch.float32):
        out = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
        _hip.check(_hip.lib().dw_fp8_cast_amax(
            _hip.ptr(x), int(x.dtype == torch.bfloat16), _hip.ptr(st.scale[idx:]), _hip.ptr(out),
            _hip.ptr(st.amax_bits[idx:]), x.numel(), int(fmt == "e5m2"), _hip.stream()), "fp8_cast_amax")
        return out.view(_TORCH_DT[fmt])
    xf = x.float()
    a = xf.abs().max() if xf.numel() else xf.new_zeros(())
    a = torch.where(torch.isnan(a), torch.full_like(a, float("inf")), a)  # as the kernels: NaN records +inf
    cur = st.amax_bits[idx: idx + 1].view(torch.float32)
    cur.copy_(torch.maximum(cur, a.reshape(1)))
    lim = FP8_MAX[fmt]
    return (xf * st.scale[idx]).clamp(-lim, lim).to(_TORCH_DT[fmt])


@torch.no_grad()
def init_scale_from(x: torch.Tensor, st: Fp8State, idx: int):
    """First use of a tensor role: its delayed-scaling history is empty, so
    set the scale from THIS tensor's amax (current scaling, device-side --
    no host sync) instead of the cold-start 1.0 that saturates or underflows
    the first step's casts (Llama-3 8B: first-step loss 11.9 vs 0.15 in bf16
    without this)."""
    a = x.detach().abs().amax().float()
    mp = float(2.0 ** st.margin)
    sc = torch.where((a > 0) & torch.isfinite(a), st.fmax[idx] / (a * mp), st.scale[idx])
    st.scale[idx] = sc
    st.inv_scale[idx] = 1.0 / sc


@torch.no_grad()
def cast_to_fp8_t(x: torch.Tensor, st: Fp8State, idx: int, fmt: str, row: bool = True, trans: bool = True):
    """x [R, C] -> (x8 [R, C] or None, x8^T [C, R] contiguous or None) in ONE
    pass (``dw_fp8_cast_t``: LDS-tiled transpose), scaled by ``st.scale[idx]``,
    amax recorded as ``cast_to_fp8``."""
    x = x.contiguous()
    R, C = x.shape
    if _hip.use_hip(x) and x.dtype in (torch.bfloat16, torch.float32) and C % 8 == 0 and R % 16 == 0:
        out = torch.empty(R, C, dtype=torch.uint8, device=x.device) if row else None
        out_t = torch.empty(C, R, dtype=torch.uint8, device=x.device) if trans else None
        _hip.check(_hip.lib().dw_fp8_cast_t(
            _hip.ptr(x), int(x.dtype == torch.bfloat16), _hip.ptr(st.scale[idx:]), _hip.ptr(out), _hip.ptr(out_t),
            _hip.ptr(st.amax_bits[idx:]), R, C, int(fmt == "e5m2"), _hip.stream()), "fp8_cast_t")
        dt = _TORCH_DT[fmt]
        return (out.view(dt) if out is not None else None), (out_t.view(dt) if out_t is not None else None)
    x8 = cast_to_fp8(x, st, idx, fmt)
    return (x8 if row else None), (x8.t().contiguous() if trans else None)


def _scaled_mm(a8, b8, inv_a, inv_b, bias, out_dtype):
    """a8 [M, K] row-major @ b8 [K, N] (column-major) with per-tensor inverse
    scales; hipBLASLt FP8 GEMM on the GPU."""
    if a8.is_cuda:
        return torch._scaled_mm(a8, b8, scale_a=inv_a, scale_b=inv_b, bias=bias, out_dtype=out_dtype)
    y = (a8.float() * inv_a) @ (b8.float() * inv_b)
    if bias is not None:
        y = y + bias.float()
    return y.to(out_dtype)


def _gemm_ok(*dims) -> bool:
    return all(d % 16 == 0 and d > 0 for d in dims)


class _Fp8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, mod):
        st = mod._state(x.device)
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16, torch.float32) else torch.bfloat16
        # x8 for this GEMM, x8^T (token dim contiguous) for the weight
        # gradient; w8 for this GEMM, w8^T for dgrad -- each from ONE pass
        need_w = weight.requires_grad
        if mod._fresh:  # first step: scales from the tensors themselves
            for i, t in ((mod._ix, x2), (mod._iw, weight)):
                if i in mod._fresh:
                    init_scale_from(t, st, i)
                    mod._fresh.discard(i)
        x8, x8t = cast_to_fp8_t(x2, st, mod._ix, "e4m3", trans=need_w)
        w8, w8t = cast_to_fp8_t(weight, st, mod._iw, "e4m3", trans=x.requires_grad)
        b = bias.to(out_dtype) if bias is not None else None
        y = _scaled_mm(x8, w8.t(), st.inv_scale[mod._ix], st.inv_scale[mod._iw], b, out_dtype)
        ctx.save_for_backward(x8t, w8t)
        ctx.mod, ctx.shape, ctx.has_bias = mod, shape, bias is not None
        ctx.wdtype, ctx.xdtype = weight.dtype, x.dtype
        return y.reshape(*shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x8t, w8t = ctx.saved_tensors
        mod = ctx.mod
        st = mod._state(gy.device)
        g2 = gy.reshape(-1, gy.shape[-1]).contiguous()
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if mod._ig in mod._fresh:
            init_scale_from(g2, st, mod._ig)
            mod._fresh.discard(mod._ig)
        # g8 for dgrad, g8^T (token dim contiguous) for the weight gradient: one pass
        g8, g8t = cast_to_fp8_t(g2, st, mod._ig, mod.grad_fmt, row=need_x, trans=need_w)
        inv_g, inv_w, inv_x = st.inv_scale[mod._ig], st.inv_scale[mod._iw], st.inv_scale[mod._ix]
        gdt = ctx.xdtype if ctx.xdtype in (torch.bfloat16, torch.float16, torch.float32) else torch.bfloat16
        dx = dw = db = None
        if need_x:
            # dx [T, in] = g [T, out] @ w [out, in]: B = w8^T viewed column-major
            dx = _scaled_mm(g8, w8t.t(), inv_g, inv_w, None, gdt).reshape(ctx.shape)
        if need_w:
            # dw [out, in] = g^T [out, T] @ x [T, in]: A = g8^T, B = x8^T viewed column-major
            wdt = ctx.wdtype if ctx.wdtype in (torch.bfloat16, torch.float16, torch.float32) else torch.float32
            dw = _scaled_mm(g8t, x8t.t(), inv_g, inv_x, None, wdt)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            if _hip.use_hip(g2) and g2.dtype == torch.bfloat16 and g2.shape[-1] % 8 == 0:
                from .activation import colsum

                db = colsum(g2, out_dtype=ctx.wdtype)  # one HIP pass, fp32 math
            else:
                db = g2.float().sum(0).to(ctx.wdtype)
        return dx, dw, db, None


class Fp8Linear(nn.Module):
    """Drop-in for ``nn.Linear`` (shares the parameters of ``linear``) whose
    GEMMs run in FP8.  Inputs whose token count is not a multiple of 16 (or
    no-grad calls of non-eligible shapes) use the bf16 path."""

    def __init__(self, linear: nn.Linear, fp8_format: str = "HYBRID"):
        super().__init__()
        self.in_features, self.out_features = linear.in_features, linear.out_features
        self.weight = linear.weight
        self.bias = linear.bias
        fmt = fp8_format.upper()
        if fmt not in ("HYBRID", "E4M3"):
            raise ValueError(f"fp8_format must be HYBRID or E4M3, not {fp8_format}")
        self.fp8_format = fmt
        self.grad_fmt = "e5m2" if fmt == "HYBRID" else "e4m3"
        self._dev = None
        self._ix = self._iw = self._ig = -1
        self._fresh = set()  # roles whose scale is still the cold-start 1.0

    def _state(self, device) -> Fp8State:
        d = torch.device(device)
        if self._dev != d:
            st = fp8_state(d)
            self._ix, self._iw, self._ig = st.register("e4m3"), st.register("e4m3"), st.register(self.grad_fmt)
            self._fresh = {self._ix, self._iw, self._ig}
            self._dev = d
        return fp8_state(d)

    def forward(self, x):
        T = x.numel() // max(1, x.shape[-1])
        if not _gemm_ok(self.in_features, self.out_features, T):
            return F.linear(x, self.weight, self.bias)
        dt = x.device.type
        if torch.is_autocast_enabled(dt):
            # outputs in the autocast dtype, as the nn.Linear it replaces
            x = x.to(torch.get_autocast_dtype(dt))
        return _Fp8LinearFn.apply(x, self.weight, self.bias, self)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, fp8_format={self.fp8_format}"


def eligible(name: str, module: nn.Module, include: Optional[Iterable[str]] = None,
             exclude: Optional[Iterable[str]] = None) -> bool:
    """The reference's include / exclude name filters plus the FP8 GEMM
    shape rule (both weight dims multiples of 16, as for the transposed
    weight of the backward)."""
    if not isinstance(module, nn.Linear):  # nn.Linear and FusedLinear (ops/linear.py)
        return False
    if exclude and any(e in name for e in exclude):
        return False
    if include is not None and not any(i in name for i in include):
        return False
    return _gemm_ok(module.in_features, module.out_features)


def replace_linears(model: nn.Module, include=None, exclude=None, fp8_format: str = "HYBRID") -> List[str]:
    """Swap every eligible ``nn.Linear`` of ``model`` for an ``Fp8Linear``
    (parameters shared, so optimizers / checkpoints see the same tensors).
    Returns the replaced names."""
    done = []
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            full = f"{name}.{cname}" if name else cname
            if eligible(full, child, include, exclude):
                setattr(mod, cname, Fp8Linear(child, fp8_format))
                done.append(full)
    return done


def fp8_stats(device=None) -> dict:
    st = fp8_state(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    n = st.n
    return {"tensors": n, "scale_min": float(st.scale[:n].min()) if n else None,
            "scale_max": float(st.scale[:n].max()) if n else None,
            "history": st.h, "steps": st.steps, "log2_margin": st.margin,
            "fmax_e4m3": FP8_MAX["e4m3"], "unit_scale": math.isclose(float(st.scale[:n].mean()), 1.0) if n else None}
