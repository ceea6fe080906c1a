"""Fused optimizers over :class:`FlatParams` (``csrc/kernels/optim.hip``).

``FusedAdamW`` / ``FusedAGD`` keep fp32 master weights (when the model is
bf16), exp_avg and exp_avg_sq as three flat fp32 buffers.  ``step()`` is one
kernel launch (plus two tiny ones for global-norm clipping, which never sync
the host: the clip coefficient stays on the device).

``state_dict()`` is torch-optimizer shaped ({"state": {idx: {...}},
"param_groups": [...]}) but every tensor in it is a view into a flat buffer,
so a flash checkpoint of the optimizer is three contiguous extents.

Parity: ATorch optimizers (atorch/atorch/optimizers/agd.py, bf16_optimizer.py,
adam_offload.py) and the fused Adam they use.
"""

import math
from typing import Optional

import torch

from ..ops import _hip
from ..parallel.flat import FlatParams


import weakref

_DEFERRING = weakref.WeakSet()  # optimizers holding a deferred state write-back


def flush_deferred_state():
    """Complete every pending deferred state write-back (device-side waits
    for the ring snapshots involved, then the replay kernels)."""
    for opt in list(_DEFERRING):
        opt.flush_deferred()


class _FlatOptimizer(torch.optim.Optimizer):
    def __init__(self, flat: FlatParams, defaults: dict, master_weights: Optional[bool] = None,
                 max_grad_norm: float = 0.0):
        self.flat = flat
        super().__init__(flat.params, defaults)
        # a lazily zeroed gradient generation (parallel/flat.py) is fully
        # defined before the update reads the whole buffer
        if hasattr(flat, "finalize_grads"):
            self.register_step_pre_hook(lambda opt, args, kwargs: opt.flat.finalize_grads())
        dev = flat.device
        self.master_weights = (flat.dtype != torch.float32) if master_weights is None else master_weights
        n = flat.numel
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.master = flat.data.float().clone() if self.master_weights else None
        # the step counter lives in a CPU tensor that the state dict exposes
        # directly: an in-place (flash checkpoint) restore restores it too
        self._step_t = torch.zeros((), dtype=torch.float32)
        self.max_grad_norm = max_grad_norm
        # e.g. 1/world for summed DDP gradients; a FlatFSDP shard brings its own
        self.grad_scale = float(getattr(flat, "grad_scale", 1.0))
        self._scalars = torch.zeros(4, dtype=torch.float32, device=dev)  # sumsq, coef, norm, pad
        self.last_grad_norm = None

    @property
    def step_count(self) -> int:
        return int(self._step_t.item())

    @step_count.setter
    def step_count(self, v: int):
        self._step_t.fill_(float(v))

    # ------------------------------------------------------------ helpers
    def _gscale_ptr(self):
        """Device scalar = grad_scale * clip coefficient (None if trivial)."""
        on_gpu = self.flat.data.is_cuda
        if self.max_grad_norm <= 0 and self.grad_scale == 1.0:
            return None
        if not on_gpu:
            return None
        L = _hip.lib()
        s = self._scalars
        if self.max_grad_norm > 0:
            s[0].zero_()
            _hip.check(L.dw_sumsq_flat(_hip.ptr(self.flat.grad), _hip.dtype_code(self.flat.grad), self.flat.numel,
                                       _hip.ptr(s[0:1]), _hip.ptr(_hip.grid_sum_ws(s.device)), _hip.stream()),
                       "sumsq")
            if getattr(self.flat, "norm_reduce", False):  # a sharded gradient (FlatFSDP): the global norm
                import torch.distributed as dist

                dist.all_reduce(s[0:1], group=self.flat.norm_group)
            _hip.check(L.dw_clip_coef(_hip.ptr(s[0:1]), float(self.max_grad_norm), float(self.grad_scale),
                                      _hip.ptr(s[1:2]), _hip.ptr(s[2:3]), _hip.stream()), "clip_coef")
            self.last_grad_norm = s[2]
        else:
            s[1].fill_(self.grad_scale)
        return s[1:2]

    def _cpu_gscale(self) -> float:
        g = self.flat.grad.float()
        scale = self.grad_scale
        if self.max_grad_norm > 0:
            sq = (g * g).sum().reshape(1)
            if getattr(self.flat, "norm_reduce", False):
                import torch.distributed as dist

                dist.all_reduce(sq, group=self.flat.norm_group)
            nrm = float(sq.sqrt()) * self.grad_scale
            self.last_grad_norm = torch.tensor(nrm)
            scale *= min(1.0, self.max_grad_norm / (nrm + 1e-6))
        return scale

    def _decay_vec(self):
        m = self.flat.decay_mask.cpu().repeat_interleave(64)[: self.flat.numel].to(self.flat.device)
        return m.bool()

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    # ------------------------------------------------- overlapped update
    _overlap = None

    def overlap_with_forward(self, model, chunks: int = 24):
        """Run each ``step()``'s update on a side stream, in forward order,
        under the next forward pass (``optimizers/overlap.py``).  Parameters
        and optimizer state are complete once that forward has returned, or
        after :meth:`join`."""
        from .overlap import StepOverlap

        if self._overlap is not None:
            self._overlap.remove()
        self._overlap = StepOverlap(self, model, chunks) if chunks > 0 else None
        return self._overlap

    def join(self):
        """Order the current stream after a pending overlapped update (and a
        deferred state write-back: the state is complete afterwards)."""
        if self._overlap is not None:
            self._overlap.join()
        self.flush_deferred()

    def _run_update(self, launch_range):
        """The update over the whole buffer: one launch, or piecewise on the
        overlap side stream."""
        if self._overlap is not None:
            self._overlap.launch(launch_range)
        else:
            launch_range(0, self.flat.numel)

    # ---------------------------- deferred state write-back (ring snapshots)
    # A flash-checkpoint snapshot through the bounded HBM ring (copier.py
    # _save_slice_ring) reads parameters and optimizer state while the next
    # forward / backward run; the next update normally has to wait until the
    # ring has taken ALL of them -- with a state larger than the ring that is
    # the PCIe drain of the excess (70B TP=8 shard: 123.5 GB, 64 GB ring,
    # ~0.7 s stall per save, profiles/r3/tp8_shard_70b_staging_ring64.json).
    # Instead the update runs at once: the elements whose state the ring has
    # copied are updated normally; for the others only the NEW PARAMETERS are
    # written (the next forward needs them) while their master / exp_avg /
    # exp_avg_sq keep the snapshot's values, and the step's gradient (+ clip
    # coefficient, lr, bias corrections) is kept.  Once the ring has drained,
    # one replay kernel applies the K kept steps and writes the state -- the
    # same per-element math (csrc/kernels/optim.hip adam_elem), so the result
    # is bit-identical to having waited.  Up to DWAMD_DEFER_STATE_STEPS
    # (default 4) steps are deferred; the memory cost is one gradient copy of
    # the deferred elements per step.  ``DWAMD_DEFER_STATE=0`` turns it off.
    _dsw = None
    _dsw_offer = None

    def offer_ring_fence(self, copier) -> bool:
        import os

        if (not self._dsw_supported() or os.environ.get("DWAMD_DEFER_STATE", "1") == "0"
                or self._overlap is not None or not self.flat.data.is_cuda):
            return False
        if self.master is None:
            # no fp32 master: the parameters ARE the weights the replay starts
            # from, and a deferred step overwrites them -- replaying the kept
            # steps would apply them twice.  Wait for the ring instead.
            return False
        if self._dsw is not None and self._dsw["copier"] is not copier:
            return False
        if self._dsw is None and not self._ring_touches(copier):
            return False  # the ring reads none of this optimizer's tensors (someone else's snapshot)
        self._dsw_offer = copier
        return True

    def _dsw_supported(self) -> bool:
        return False

    def _ring_touches(self, copier) -> bool:
        f = self.flat
        mine = [(f.data.data_ptr(), f.data.data_ptr() + f.data.element_size() * f.numel)] + self._dsw_ranges(
            0, f.numel)
        return any(a < mb and ma < b for a, b in copier.ring_sources() for ma, mb in mine)

    def _dsw_ranges(self, lo: int, hi: int):
        out = []
        for t, es in ((self.exp_avg, 4), (self.exp_avg_sq, 4), (self.master, 4)):
            if t is not None:
                out.append((t.data_ptr() + es * lo, t.data_ptr() + es * hi))
        return out

    def _dsw_first_unstaged(self, copier) -> int:
        """First flat element whose state the ring reads but has not copied
        yet (flat.numel: none)."""
        src, staged = copier.ring_sources(), copier.ring_staged()
        n = self.flat.numel
        first = n
        for t in (self.exp_avg, self.exp_avg_sq, self.master):
            if t is None:
                continue
            base, end = t.data_ptr(), t.data_ptr() + 4 * n
            # the part of the buffer the snapshot covers, minus what it has copied
            for a, b in src:
                a, b = max(a, base), min(b, end)
                if a >= b:
                    continue
                cur = a
                for sa, sb in staged:
                    if sa <= cur < sb:
                        cur = sb
                if cur < b:
                    first = min(first, (cur - base) // 4)
                    break
        return first

    def _dsw_replay(self, write_state: bool, extra=None):
        """Launch the replay over the deferred elements: the kept steps (+
        ``extra`` = this step's (grad view, gscale, lr, bc1, bc2))."""
        import ctypes

        d = self._dsw
        lo, f = d["lo"], self.flat
        n = f.numel - lo
        steps = list(d["steps"]) + ([extra] if extra is not None else [])
        K = len(steps)
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        arr = ctypes.c_void_p * K
        farr = ctypes.c_float * K
        grads = arr(*[ctypes.c_void_p(x[0].data_ptr()) for x in steps])
        gss = arr(*[ctypes.c_void_p(x[1].data_ptr() if x[1] is not None else 0) for x in steps])
        ms = self.master
        _hip.check(_hip.lib().dw_adam_replay(
            _hip.ptr(f.data[lo:]), _hip.dtype_code(f.data), _hip.ptr(None if ms is None else ms[lo:]),
            _hip.ptr(self.exp_avg[lo:]), _hip.ptr(self.exp_avg_sq[lo:]), n, K, grads, _hip.dtype_code(f.grad), gss,
            farr(*[x[2] for x in steps]), farr(*[x[3] for x in steps]), farr(*[x[4] for x in steps]), float(b1),
            float(b2), float(g["eps"]), float(g["weight_decay"]), int(getattr(self, "adamw", True)),
            _hip.ptr(f.decay_mask[lo // 64:]), int(write_state), _hip.stream()), "adam_replay")

    def flush_deferred(self):
        """Write the deferred state back: the current stream waits for the
        ring snapshot (device side), then the replay runs on it."""
        d = self._dsw
        if d is None:
            return
        c = d["copier"]
        c.fence()  # every chunk copied: the old state may be overwritten now
        from ..flash_checkpoint import copier as _cp

        if _cp._FENCED is not None:
            _cp._FENCED.discard(c)
        self._dsw_replay(True)
        self._dsw = None
        _DEFERRING.discard(self)

    def _dsw_step(self, launch, gs, lr, bc1, bc2) -> bool:
        """The update under a pending ring snapshot (see above).  Returns
        False when no deferral applies (the caller runs the plain update)."""
        import os

        c = self._dsw_offer
        self._dsw_offer = None
        if c is None:
            return False
        f = self.flat
        n = f.numel
        from ..flash_checkpoint import copier as _cp

        def discard():
            if _cp._FENCED is not None:
                _cp._FENCED.discard(c)

        if c.ring_done():
            # drained: complete any deferral, then the plain update
            if self._dsw is not None:
                self.flush_deferred()
            c.fence()
            discard()
            return False
        if self._dsw is None:
            lo = self._dsw_first_unstaged(c) // 256 * 256
            if lo >= n:  # the state is fully copied; only parameters may still be in flight
                c.ring_wait_ranges([(f.data.data_ptr(), f.data.data_ptr() + f.data.element_size() * n)])
                return False
            kmax = self._defer_budget((n - lo) * f.grad.element_size())
            if kmax < 1:
                # not even one kept gradient fits next to the next step's
                # activations: wait for the ring (the stall deferral avoids)
                c.fence()
                discard()
                return False
            self._dsw = {"copier": c, "lo": lo, "steps": [], "kmax": kmax}
            _DEFERRING.add(self)
        d = self._dsw
        kmax = d["kmax"]
        if len(d["steps"]) >= kmax:
            self.flush_deferred()  # waits for the ring (the stall this bounds)
            c.fence()
            discard()
            return False
        lo = d["lo"]
        # parameters are written below: their snapshot copies must have run
        c.ring_wait_ranges([(f.data.data_ptr(), f.data.data_ptr() + f.data.element_size() * n)])
        if lo > 0:
            launch(0, lo)  # staged state: the plain update
        gk = f.grad[lo:].clone()  # this step's gradient of the deferred elements
        gsk = gs.clone() if gs is not None else None
        step = (gk, gsk, float(lr), float(bc1), float(bc2))
        self._dsw_replay(False, extra=step)  # new parameters from the snapshot's state + the kept steps
        d["steps"].append(step)
        return True

    last_defer_plan = None

    def _defer_budget(self, per_step: int) -> int:
        """Deferred steps (K) whose kept gradients fit in HBM: each deferred
        step keeps a copy of the deferred elements' gradient until the ring
        drains.  Budget = the driver's free HBM minus ``DWAMD_DEFER_RESERVE_GB``
        (2).  The caching allocator's unused cache is NOT counted: at an
        optimizer step it holds the blocks the freed activations came from,
        which the next forward takes again (a process-lifetime peak statistic
        is no measure of that: it keeps earlier, larger workloads).  K =
        min(DWAMD_DEFER_STATE_STEPS, 4 by default, budget // per-step
        bytes); 0 = wait for the ring.  The plan is kept in
        ``last_defer_plan`` (and counted by ``hbm_budget.plan``'s
        ``defer_bytes``)."""
        import os

        kcap = max(1, min(7, int(os.environ.get("DWAMD_DEFER_STATE_STEPS", "4"))))
        dev = self.flat.device
        try:
            free = int(torch.cuda.mem_get_info(dev)[0])
            cached = max(0, int(torch.cuda.memory_reserved(dev)) - int(torch.cuda.memory_allocated(dev)))
        except Exception:
            free, cached = 0, 0
        margin = int(float(os.environ.get("DWAMD_DEFER_RESERVE_GB", "2")) * (1 << 30))
        budget = free - margin
        k = max(0, min(kcap, budget // max(1, per_step + 64)))
        self.last_defer_plan = {"steps": int(k), "per_step_bytes": int(per_step), "budget_bytes": int(budget),
                                "driver_free_bytes": int(free), "allocator_cache_bytes": int(cached),
                                "decision": "defer" if k >= 1 else "wait"}
        from ..common.log import logger

        logger.info(f"deferred optimizer-state write-back plan: {self.last_defer_plan}")
        return int(k)

    def checkpoint_safe_tensors(self):
        """Tensors only ``step()`` writes (an overlapped flash-checkpoint
        snapshot may still be reading them after the save call returns)."""
        return [t for t in (self.flat.data, self.exp_avg, self.exp_avg_sq, self.master) if t is not None]

    # -------------------------------------------------------- state dict
    def state_dict(self):
        self.flush_deferred()
        # The per-parameter views never change: build them once.  All params
        # share one "step" tensor (same value), updated in place.
        if getattr(self, "_sd_views", None) is None:
            views = {}
            for i, (o, c) in enumerate(self.flat.offsets):
                p = self.flat.params[i]
                v = {"exp_avg": self.exp_avg[o:o + c].view(p.shape),
                     "exp_avg_sq": self.exp_avg_sq[o:o + c].view(p.shape)}
                if self.master is not None:
                    v["master_param"] = self.master[o:o + c].view(p.shape)
                views[i] = v
            self._sd_views = views
        state = {i: {"step": self._step_t, **v} for i, v in self._sd_views.items()}
        groups = []
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(len(self.flat.params)))
            groups.append(d)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        self.flush_deferred()
        st = sd["state"]
        if self.exp_avg.is_cuda:
            # a flash-checkpoint restore may still be landing this state on a
            # side stream (deferred_restore.py): order these copies after it
            from ..flash_checkpoint import deferred_restore

            deferred_restore.wait_all()

        def put(dst, src):
            src = src.reshape(-1)
            if src.data_ptr() == dst.data_ptr() and src.numel() == dst.numel() and src.dtype == dst.dtype:
                return  # the restore wrote these views in place already
            dst.copy_(src)

        with torch.no_grad():
            for i, (o, c) in enumerate(self.flat.offsets):
                if i not in st:
                    continue
                s = st[i]
                put(self.exp_avg[o:o + c], s["exp_avg"])
                put(self.exp_avg_sq[o:o + c], s["exp_avg_sq"])
                if self.master is not None and "master_param" in s:
                    put(self.master[o:o + c], s["master_param"])
                self.step_count = int(float(s["step"]))
        for g, sg in zip(self.param_groups, sd.get("param_groups", [])):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v


class FusedAdamW(_FlatOptimizer):
    def __init__(self, flat: FlatParams, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                 adamw=True, master_weights=None, max_grad_norm=0.0):
        super().__init__(flat, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay), master_weights,
                         max_grad_norm)
        self.adamw = adamw

    def _dsw_supported(self) -> bool:
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.step_count += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        f = self.flat
        if f.data.is_cuda:
            if self._overlap is not None:
                self._overlap.join()  # the previous update, if no forward ran since
            gs = self._gscale_ptr()
            ms = self.master

            def launch(lo, hi):
                _hip.check(_hip.lib().dw_adam_flat(
                    _hip.ptr(f.data[lo:hi]), _hip.dtype_code(f.data), _hip.ptr(None if ms is None else ms[lo:hi]),
                    _hip.ptr(f.grad[lo:hi]), _hip.dtype_code(f.grad), _hip.ptr(self.exp_avg[lo:hi]),
                    _hip.ptr(self.exp_avg_sq[lo:hi]), _hip.ptr(gs), hi - lo, 0, float(g["lr"]), float(b1),
                    float(b2), float(g["eps"]), float(g["weight_decay"]), float(bc1), float(bc2), int(self.adamw),
                    _hip.ptr(f.decay_mask[lo // 64:]), _hip.stream()), "adam")

            if self._dsw_offer is not None and self._dsw_step(launch, gs, g["lr"], bc1, bc2):
                return loss
            if self._dsw is not None:
                self.flush_deferred()  # (a fence taken over earlier, no longer offered)
            self._run_update(launch)
            return loss
        # CPU path (reference math)
        scale = self._cpu_gscale()
        grad = f.grad.float() * scale
        w = self.master if self.master is not None else f.data
        decay = self._decay_vec()
        lr, wd, eps = g["lr"], g["weight_decay"], g["eps"]
        if not self.adamw and wd:
            grad = grad + wd * w * decay
        self.exp_avg.mul_(b1).add_(grad, alpha=1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1 - b2)
        denom = self.exp_avg_sq.sqrt() / math.sqrt(bc2) + eps
        if self.adamw and wd:
            w.sub_(lr * wd * w * decay)
        w.addcdiv_(self.exp_avg, denom, value=-lr / bc1)
        if self.master is not None:
            f.data.copy_(w.to(f.data.dtype))
        return loss


class FusedAGD(_FlatOptimizer):
    """AGD (reference atorch/atorch/optimizers/agd.py) on flat buffers."""

    def __init__(self, flat: FlatParams, lr=1e-3, betas=(0.9, 0.999), delta=1e-5, weight_decay=0.0,
                 clip=None, master_weights=None, max_grad_norm=0.0):
        super().__init__(flat, dict(lr=lr, betas=betas, delta=delta, weight_decay=weight_decay, clip=clip),
                         master_weights, max_grad_norm)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.step_count += 1
        t = self.step_count
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
        bc1_prev = 1.0 - b1 ** (t - 1) if t > 1 else 0.0
        clip = float(g["clip"]) if g["clip"] is not None else 0.0
        f = self.flat
        if f.data.is_cuda:
            if self._overlap is not None:
                self._overlap.join()
            gs = self._gscale_ptr()
            ms = self.master

            def launch(lo, hi):
                _hip.check(_hip.lib().dw_agd_flat(
                    _hip.ptr(f.data[lo:hi]), _hip.dtype_code(f.data), _hip.ptr(None if ms is None else ms[lo:hi]),
                    _hip.ptr(f.grad[lo:hi]), _hip.dtype_code(f.grad), _hip.ptr(self.exp_avg[lo:hi]),
                    _hip.ptr(self.exp_avg_sq[lo:hi]), _hip.ptr(gs), hi - lo, 0, float(g["lr"]), float(b1),
                    float(b2), float(g["delta"]), float(g["weight_decay"]), float(bc1), float(bc1_prev), float(bc2),
                    clip, _hip.ptr(f.decay_mask[lo // 64:]), _hip.stream()), "agd")

            self._run_update(launch)
            return loss
        scale = self._cpu_gscale()
        grad = f.grad.float() * scale
        w = self.master if self.master is not None else f.data
        decay = self._decay_vec()
        lr, wd = g["lr"], g["weight_decay"]
        if wd:
            w.mul_(torch.where(decay, 1.0 - lr * wd, 1.0))
        m_old = self.exp_avg.clone()
        self.exp_avg.mul_(b1).add_(grad, alpha=1 - b1)
        upd = self.exp_avg / bc1 if t == 1 else self.exp_avg / bc1 - m_old / bc1_prev
        self.exp_avg_sq.mul_(b2).addcmul_(upd, upd, value=1 - b2)
        den = self.exp_avg_sq.sqrt().clamp(min=g["delta"] * math.sqrt(bc2))
        u = self.exp_avg / den
        if clip:
            u.clamp_(-clip, clip)
        w.add_(u, alpha=-lr * math.sqrt(bc2) / bc1)
        if self.master is not None:
            f.data.copy_(w.to(f.data.dtype))
        return loss
