"""Multi-tensor fused AdamW / AGD over arbitrary parameter lists
(``csrc/kernels/optim_multi.hip``).

:class:`~dlrover_wuqiong_amd.optimizers.fused.FusedAdamW` needs the model's
parameters packed into one :class:`FlatParams` buffer.  Under FSDP2, tensor
parallelism or plain DDP the parameters live where those wrappers put them
(DTensor local shards, per-parameter storages), so these optimizers take any
``params`` iterable like ``torch.optim.AdamW`` and still update all of them in
ONE HIP launch: a device table of per-tensor descriptors (param / grad /
master / moment pointers) plus a chunk table that the workgroups grid-stride
over.  The descriptor table is re-uploaded only when a gradient pointer moves.

State layout (what a flash checkpoint copies): the fp32 ``exp_avg``,
``exp_avg_sq`` and -- for bf16 parameters -- ``master_param`` of every
parameter are views into three flat per-device buffers, so the optimizer
state is three contiguous extents.  ``state[p]`` holds those views (wrapped
as DTensors with the parameter's mesh/placements for DTensor parameters), so
``optimizer.state_dict()``, ``torch.distributed.checkpoint`` and
``get_state_dict`` see the standard torch layout; ``load_state_dict`` copies
into the views instead of replacing them.

bf16 parameters + fp32 masters is ATorch's "half + BF16Optimizer" recipe
(atorch/atorch/optimizers/bf16_optimizer.py): FSDP2 then all-gathers bf16
directly (no per-step fp32->bf16 cast kernels) and the update writes the
bf16 copy from the fp32 master in the same pass.

Global-norm gradient clipping (``max_grad_norm``) runs on the device: a
multi-tensor sum-of-squares kernel, one all-reduce of a scalar for sharded
(DTensor) parameters, and a clip coefficient the update kernel reads -- no
host synchronisation.

Parity: torch.optim.AdamW/Adam math; AGD as reference
atorch/atorch/optimizers/agd.py:84-150 (decoupled, non-fixed decay).
"""

import ctypes
import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..ops import _hip

_DESC = np.dtype([("p", "<u8"), ("g", "<u8"), ("master", "<u8"), ("m", "<u8"), ("v", "<u8"), ("n", "<i8"),
                  ("flags", "<i4"), ("group", "<i4"), ("norm_w", "<f4"), ("pad", "<i4")])
assert _DESC.itemsize == 64
MAX_GROUPS = 16
_ALIGN = 64  # elements: every state view starts 256 B aligned
_HYPER_FIELDS = ("lr", "wd", "b1", "b2", "eps", "bc1", "bc2", "bc1_prev", "clip")


def _is_dtensor(t) -> bool:
    return hasattr(t, "_local_tensor") and hasattr(t, "device_mesh")


def _local(t: torch.Tensor) -> torch.Tensor:
    return t._local_tensor if _is_dtensor(t) else t


def _wrap_like(view: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    if _is_dtensor(p):
        from torch.distributed.tensor import DTensor

        return DTensor.from_local(view, p.device_mesh, p.placements, run_check=False, shape=p.shape,
                                  stride=p.stride())
    return view


def _replicate_factor(p) -> float:
    if not _is_dtensor(p):
        return 1.0
    f = 1
    for i, pl in enumerate(p.placements):
        if pl.is_replicate():
            f *= p.device_mesh.size(i)
    return float(f)


class _MultiTensorOptimizer(torch.optim.Optimizer):
    _agd = False

    def __init__(self, params, defaults: dict, master_weights: Optional[bool], max_grad_norm: float,
                 grad_scale: float):
        super().__init__(params, defaults)
        if len(self.param_groups) > MAX_GROUPS:
            raise ValueError(f"at most {MAX_GROUPS} param groups (got {len(self.param_groups)})")
        self.max_grad_norm = float(max_grad_norm or 0.0)
        self.grad_scale = float(grad_scale)
        self.last_grad_norm = None
        self._step_t = torch.zeros((), dtype=torch.float32)  # shared by every param's state["step"]
        self._master_weights = master_weights
        self._table_cache = {}  # slot -> (key, tables): the whole step, or per FSDP unit (in_backward.py)
        self._in_backward = None
        self._build_state()

    # ------------------------------------------------------------ state
    @property
    def step_count(self) -> int:
        return int(self._step_t.item())

    def _all_params(self) -> List[torch.Tensor]:
        return [p for g in self.param_groups for p in g["params"]]

    def _build_state(self):
        per_dev: Dict[torch.device, List[torch.Tensor]] = {}
        for p in self._all_params():
            loc = _local(p)
            if not loc.is_contiguous():
                raise ValueError("multi-tensor optimizer needs contiguous (local) parameters")
            per_dev.setdefault(loc.device, []).append(p)
        self._flat = {}
        for dev, ps in per_dev.items():
            sizes = [(_local(p).numel() + _ALIGN - 1) // _ALIGN * _ALIGN for p in ps]
            total = max(1, sum(sizes))
            need_master = any(self._wants_master(p) for p in ps)
            bufs = {"exp_avg": torch.zeros(total, dtype=torch.float32, device=dev),
                    "exp_avg_sq": torch.zeros(total, dtype=torch.float32, device=dev)}
            if need_master:
                bufs["master_param"] = torch.zeros(total, dtype=torch.float32, device=dev)
            self._flat[dev] = bufs
            off = 0
            for p, sz in zip(ps, sizes):
                loc = _local(p)
                n = loc.numel()
                st = {"step": self._step_t}
                for k, buf in bufs.items():
                    if k == "master_param" and not self._wants_master(p):
                        continue
                    view = buf[off:off + n].view(loc.shape)
                    if k == "master_param":
                        with torch.no_grad():
                            view.copy_(loc.detach().float())
                    st[k] = _wrap_like(view, p)
                self.state[p] = st
                off += sz

    def _wants_master(self, p) -> bool:
        if self._master_weights is False:
            return False
        return _local(p).dtype != torch.float32

    def flat_state_buffers(self):
        """{device: {"exp_avg": t, "exp_avg_sq": t[, "master_param": t]}}"""
        return self._flat

    def load_state_dict(self, state_dict):
        """Copy into the existing state views (the flat layout is kept)."""
        params = self._all_params()
        st = state_dict["state"]
        with torch.no_grad():
            for i, p in enumerate(params):
                s = st.get(i)
                if s is None:
                    continue
                mine = self.state[p]
                for k, v in s.items():
                    if k == "step":
                        self._step_t.fill_(float(v))
                        continue
                    if k not in mine:
                        continue
                    dst, src = _local(mine[k]), _local(v) if isinstance(v, torch.Tensor) else v
                    if isinstance(src, torch.Tensor):
                        if dst.data_ptr() != src.data_ptr():
                            dst.copy_(src.reshape(dst.shape))
        for g, sg in zip(self.param_groups, state_dict.get("param_groups", [])):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v

    # ------------------------------------------------------------ step
    def _hyper(self) -> dict:
        t = self.step_count
        h = {k: np.zeros(MAX_GROUPS, dtype=np.float32) for k in _HYPER_FIELDS}
        for gi, g in enumerate(self.param_groups):
            b1, b2 = g["betas"]
            h["lr"][gi] = g["lr"]
            h["wd"][gi] = g["weight_decay"]
            h["b1"][gi], h["b2"][gi] = b1, b2
            h["eps"][gi] = g["delta"] if self._agd else g["eps"]
            h["bc1"][gi] = 1.0 - b1 ** t
            h["bc2"][gi] = 1.0 - b2 ** t
            h["bc1_prev"][gi] = (1.0 - b1 ** (t - 1)) if t > 1 else 0.0
            h["clip"][gi] = float(g.get("clip") or 0.0) if self._agd else 0.0
        return h

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        ib = self._in_backward
        if ib is not None and ib.owns_step():
            ib.finish()  # the backward ran this step's update per FSDP unit (optimizers/in_backward.py)
            return loss
        self._step_t += 1
        live = [(gi, p) for gi, g in enumerate(self.param_groups) for p in g["params"] if p.grad is not None]
        if not live:
            return loss
        if _local(live[0][1]).is_cuda:
            self._cuda_step(live)
        else:
            self._cpu_step(live)
        return loss

    # ---- GPU: one multi-tensor launch (+ two tiny ones when clipping)
    def _tables_for(self, live, slot=None):
        key = tuple((gi, _local(p.grad).data_ptr(), _local(p).data_ptr()) for gi, p in live)
        hit = self._table_cache.get(slot)
        if hit is not None and hit[0] == key:
            return hit[1]
        L = _hip.lib()
        chunk = int(L.dw_mt_chunk())
        desc = np.zeros(len(live), dtype=_DESC)
        chunks = []
        for ti, (gi, p) in enumerate(live):
            loc, g = _local(p), _local(p.grad)
            if g.dtype not in (torch.float32, torch.bfloat16) or loc.dtype not in (torch.float32, torch.bfloat16):
                raise TypeError(f"multi-tensor optimizer: unsupported dtypes {loc.dtype}/{g.dtype}")
            if not g.is_contiguous() or g.shape != loc.shape:
                raise ValueError("multi-tensor optimizer needs contiguous grads shaped like the (local) param")
            st = self.state[p]
            m, v = _local(st["exp_avg"]), _local(st["exp_avg_sq"])
            ma = _local(st["master_param"]) if "master_param" in st else None
            ptrs = [loc.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()] + ([ma.data_ptr()] if ma is not None
                                                                                   else [])
            aligned = all(x % 16 == 0 for x in ptrs)
            n = loc.numel()
            desc[ti] = (loc.data_ptr(), g.data_ptr(), ma.data_ptr() if ma is not None else 0, m.data_ptr(),
                        v.data_ptr(), n, (1 if loc.dtype == torch.bfloat16 else 0)
                        | (2 if g.dtype == torch.bfloat16 else 0) | (4 if aligned else 0), gi,
                        1.0 / _replicate_factor(p), 0)
            nch = (n + chunk - 1) // chunk
            if nch:
                chunks.append(np.stack([np.full(nch, ti, dtype=np.int32), np.arange(nch, dtype=np.int32)], 1))
        ch = np.concatenate(chunks) if chunks else np.zeros((0, 2), dtype=np.int32)
        dev = _local(live[0][1]).device
        d_desc = torch.from_numpy(desc.view(np.uint8).copy()).pin_memory().to(dev, non_blocking=True)
        d_chunks = torch.from_numpy(np.ascontiguousarray(ch).view(np.uint8).reshape(-1)).pin_memory().to(
            dev, non_blocking=True)
        sharded = any(_is_dtensor(p) for _gi, p in live)
        tables = (d_desc, d_chunks, len(ch), sharded)
        self._table_cache[slot] = (key, tables)
        return tables

    def _cuda_step(self, live, slot=None, max_blocks: int = 0):
        L = _hip.lib()
        d_desc, d_chunks, nchunks, sharded = self._tables_for(live, slot)
        dev = d_desc.device
        gs = None
        if self.max_grad_norm > 0 or self.grad_scale != 1.0:
            s = getattr(self, "_scalars", None)
            if s is None or s.device != dev:
                s = self._scalars = torch.zeros(4, dtype=torch.float32, device=dev)
            if self.max_grad_norm > 0:
                s[0].zero_()
                _hip.check(L.dw_mt_sumsq(_hip.ptr(d_desc), _hip.ptr(d_chunks), nchunks, _hip.ptr(s[0:1]),
                                         _hip.ptr(_hip.grid_sum_ws(dev)), _hip.stream()), "mt_sumsq")
                if sharded and dist.is_initialized() and dist.get_world_size() > 1:
                    dist.all_reduce(s[0:1])
                _hip.check(L.dw_clip_coef(_hip.ptr(s[0:1]), float(self.max_grad_norm), float(self.grad_scale),
                                          _hip.ptr(s[1:2]), _hip.ptr(s[2:3]), _hip.stream()), "clip_coef")
                self.last_grad_norm = s[2]
            else:
                s[1].fill_(self.grad_scale)
            gs = s[1:2]
        h = self._hyper()
        raw = np.concatenate([h[k] for k in _HYPER_FIELDS] + [np.array([1 if self._adamw_flag() else 0],
                                                                          dtype=np.int32).view(np.float32)])
        assert raw.nbytes == int(L.dw_mt_hyper_size()), "MTHyper layout mismatch"
        _hip.check(L.dw_mt_adam_grid(_hip.ptr(d_desc), _hip.ptr(d_chunks), nchunks, _hip.ptr(gs),
                                     ctypes.c_void_p(raw.ctypes.data), int(self._agd), int(max_blocks),
                                     _hip.stream()), "mt_step")

    def _adamw_flag(self) -> bool:
        return True

    # ---- CPU: reference math (gloo path, numerics oracle)
    def _cpu_scale(self, live) -> float:
        scale = self.grad_scale
        if self.max_grad_norm > 0:
            sq = torch.zeros((), dtype=torch.float64)
            for _gi, p in live:
                sq += _local(p.grad).double().pow(2).sum() / _replicate_factor(p)
            if any(_is_dtensor(p) for _gi, p in live) and dist.is_initialized() and dist.get_world_size() > 1:
                dist.all_reduce(sq)
            nrm = math.sqrt(float(sq)) * self.grad_scale
            self.last_grad_norm = torch.tensor(nrm)
            scale *= min(1.0, self.max_grad_norm / (nrm + 1e-6))
        return scale

    def _cpu_step(self, live):
        scale = self._cpu_scale(live)
        t = self.step_count
        for gi, p in live:
            g = self.param_groups[gi]
            st = self.state[p]
            loc = _local(p)
            w = _local(st["master_param"]) if "master_param" in st else loc
            grad = _local(p.grad).float() * scale
            m, v = _local(st["exp_avg"]), _local(st["exp_avg_sq"])
            self._cpu_update(g, t, grad, w, m, v)
            if w is not loc:
                loc.copy_(w.to(loc.dtype))


class MultiTensorAdamW(_MultiTensorOptimizer):
    """``torch.optim.AdamW`` (``adamw=True``) / ``Adam`` (``adamw=False``)
    in one HIP launch over any parameter list."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, adamw=True,
                 master_weights=None, max_grad_norm=0.0, grad_scale=1.0, amsgrad=False, maximize=False,
                 foreach=None, fused=None, capturable=False, differentiable=False):
        if amsgrad or maximize or differentiable:
            raise ValueError("MultiTensorAdamW: amsgrad / maximize / differentiable are not supported")
        if isinstance(lr, torch.Tensor):
            lr = float(lr)
        self.adamw = adamw
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay),
                         master_weights, max_grad_norm, grad_scale)

    def _adamw_flag(self) -> bool:
        return self.adamw

    def _cpu_update(self, g, t, grad, w, m, v):
        b1, b2 = g["betas"]
        lr, wd, eps = g["lr"], g["weight_decay"], g["eps"]
        bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
        if not self.adamw and wd:
            grad = grad + wd * w
        m.mul_(b1).add_(grad, alpha=1 - b1)
        v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
        denom = v.sqrt() / math.sqrt(bc2) + eps
        if self.adamw and wd:
            w.mul_(1.0 - lr * wd)
        w.addcdiv_(m, denom, value=-lr / bc1)


class MultiTensorAGD(_MultiTensorOptimizer):
    """AGD (reference atorch/atorch/optimizers/agd.py) in one HIP launch."""

    _agd = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), delta=1e-5, weight_decay=0.0, clip=None,
                 master_weights=None, max_grad_norm=0.0, grad_scale=1.0, weight_decouple=True, fixed_decay=False,
                 amsgrad=False, win=False):
        if not weight_decouple or fixed_decay or amsgrad or win:
            raise ValueError("MultiTensorAGD: only the decoupled, non-fixed-decay AGD variant is fused")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), delta=delta, weight_decay=weight_decay, clip=clip),
                         master_weights, max_grad_norm, grad_scale)

    def _cpu_update(self, g, t, grad, w, m, v):
        b1, b2 = g["betas"]
        lr, wd = g["lr"], g["weight_decay"]
        bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
        if wd:
            w.mul_(1.0 - lr * wd)
        m_old = m.clone()
        m.mul_(b1).add_(grad, alpha=1 - b1)
        s = m / bc1 if t == 1 else m / bc1 - m_old / (1.0 - b1 ** (t - 1))
        v.mul_(b2).addcmul_(s, s, value=1 - b2)
        den = v.sqrt().clamp(min=g["delta"] * math.sqrt(bc2))
        u = m / den
        if g["clip"]:
            u.clamp_(-g["clip"], g["clip"])
        w.add_(u, alpha=-lr * math.sqrt(bc2) / bc1)


def fused_equivalent(optim_cls, optim_args: dict):
    """The multi-tensor fused class replacing a torch / ATorch optimizer class
    (``None`` if the requested variant has no fused kernel)."""
    from .agd import AGD

    args = dict(optim_args or {})
    if optim_cls in (torch.optim.AdamW, torch.optim.Adam):
        if args.get("amsgrad") or args.get("maximize") or args.get("differentiable"):
            return None, args
        args["adamw"] = optim_cls is torch.optim.AdamW
        if optim_cls is torch.optim.Adam:
            args.setdefault("weight_decay", 0.0)
        return MultiTensorAdamW, args
    if optim_cls is AGD:
        if args.get("amsgrad") or args.get("win") or args.get("fixed_decay") or args.get("weight_decouple") is False:
            return None, args
        return MultiTensorAGD, args
    return None, args
