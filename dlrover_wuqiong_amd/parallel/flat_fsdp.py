"""Flat-unit FSDP (ZeRO-3 / ZeRO-2) whose collectives read and write the
parameters and gradients in place.

torch FSDP2 keeps every parameter as its own dim-0 shard.  Each all-gather
therefore copies the unit's shards into one input buffer (``_foreach_copy_``),
gathers, and copies every parameter back out of the rank-interleaved output
(``split_with_sizes_copy``); each reduce-scatter first packs the gradients
with ``chunk_cat``.  On the Llama-3-8B step (1 GPU, no resharding) those
copies are 30 ms of ``copyBuffer`` + 6 ms of ``chunk_cat`` per 242 ms step
(``profiles/r5/llama3_8b_fsdp_half_noac_kernels.md``) -- a full extra
read + write of the model, twice, at HBM speed.

Here a unit (one ``wrap_cls`` module, e.g. a decoder layer; the root owns
the parameters outside every unit) is ONE flat buffer:

* the unit's parameters are views of ``full`` (each on a 64-element
  boundary, the buffer padded to a multiple of world x 64); rank r owns the
  contiguous slice ``[r L, (r + 1) L)``.  Every unit's slice lives in one
  per-rank shard buffer (``shard_flat``), which is what the fused optimizer
  updates (one streaming kernel, ``optimizers/fused.py``, fp32 masters and
  clipping over the global norm);
* ``all_gather_into_tensor(full, shard)`` writes the parameters in place --
  no copy in, no copy out; gradients are views of one flat ``gfull`` and
  ``reduce_scatter_tensor(shard_grad, gfull)`` reads them in place (summed;
  the optimizer applies 1/world inside its update);
* the fused ops write gradients straight into those views with lazy zeroing
  (``parallel/flat.py`` ``claim``), so no memset either;
* world 1: ``full`` IS the shard and ``gfull`` the shard gradient -- no
  extra buffer, no collective, no hook;
* ``reshard_after_forward`` (ZeRO-3): a unit's storage is released after its
  forward and re-gathered when its backward starts (the storage-resize trick
  of FSDP: saved tensors are views of the same storage); the next unit's
  gather is prefetched (forward order recorded by the first forward, reverse
  order in backward).  ZeRO-3 also gives a layer's unsharded gradient buffer
  back once its reduce-scatter has completed and takes it again when the
  layer's backward starts, so neither full-size buffer outlives its use
  (``p.grad`` of a wrapped parameter is then only valid inside the backward:
  the gradient is the shard's, ``shard_flat.grad``; clip through the
  optimizer's ``max_grad_norm``).  Without resharding (ZeRO-2) the gathered
  parameters and the unsharded gradients stay, as in DDP.  The root stays
  gathered.

Readiness of a unit's gradient is counted like ``FlatDDP``'s buckets: the
first backward records how often each parameter's post-accumulate hook
fires and reduces everything at the end; later backwards reduce a unit as
soon as all of its calls have arrived, overlapping the rest of the backward.

Checkpoints (``atorch/fsdp_flat_ckpt.py``) store each rank's element range
of every flattened parameter -- ATorch's FSDP FlatParameter shard format
(reference atorch/atorch/utils/fsdp_save_util.py ``save_fsdp_flat_param``:
a flat_param shard plus per-parameter offsets), readable at any world size.

Parity: reference ATorch shards with torch FSDP1 FlatParameter units
(atorch/atorch/auto/opt_lib/zero_optimization.py ``FSDPOptimization``,
``data_parallel/zero_ddp_mix_112.py``); this is the same unit structure,
built on RCCL's in-place tensor collectives instead.
"""

from contextlib import contextmanager
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ..common.log import logger
from .flat import ALIGN, FlatParams, default_no_decay


class _Unit:
    __slots__ = ("idx", "module", "flat", "full", "gfull", "shard", "shard_grad", "base", "lo", "len", "work",
                 "fresh", "released", "rs_work", "nbytes", "is_root", "names", "reduced", "grad_released")

    def __init__(self, idx, module, is_root):
        self.idx, self.module, self.is_root = idx, module, is_root
        self.work = self.rs_work = None
        self.fresh = False  # ``full`` holds the current shards' values
        self.released = False
        self.reduced = False  # reduce-scatter launched in this backward
        self.grad_released = False  # ``gfull``'s storage given back (ZeRO-3)


class ShardFlat:
    """The rank's shard of every unit, back to back, shaped like a
    ``FlatParams`` for the fused optimizers (``_FlatOptimizer``): one
    parameter (the whole shard), its gradient, the weight-decay mask, and
    ``norm_group`` so gradient clipping sums the squared norm over ranks."""

    def __init__(self, owner: "FlatFSDP", data: torch.Tensor, grad: torch.Tensor, decay_mask: torch.Tensor):
        self._owner = owner
        self.data, self.grad = data, grad
        self.numel = data.numel()
        self.dtype, self.grad_dtype, self.device = data.dtype, grad.dtype, data.device
        self.param = nn.Parameter(data, requires_grad=True)
        self.param.grad = grad
        self.params = [self.param]
        self.names = ["flat_shard"]
        self.offsets = [(0, self.numel)]
        self.decay_mask = decay_mask
        self.norm_reduce = owner.world > 1  # over norm_group (None: the default group)
        self.norm_group = owner.pg
        self.grad_scale = 1.0 / (owner.world * owner.replicas)

    def finalize_grads(self):
        self._owner.finish_gradient_sync()

    def zero_grad(self):
        self._owner.zero_grad()


class FlatFSDP(nn.Module):
    def __init__(self, module: nn.Module, wrap_cls: Sequence[type] = (), process_group=None,
                 reshard_after_forward: bool = True, prefetch: bool = True,
                 no_decay_fn: Callable[[str, torch.Tensor], bool] = default_no_decay,
                 sync_module_states: bool = True, device=None, init_seed: int = 0,
                 buffer_init_fn: Optional[Callable] = None, replicate_group=None):
        """A ``module`` built on the meta device (``torch.device("meta")``)
        is materialised per shard: each rank allocates only its shard (and,
        without resharding, the unit buffers it gathers into) on ``device``
        and fills its element range of every parameter from the sharding-
        invariant counter-based streams of ``atorch/meta_init.py``
        (``init_spec`` of the model, else the module type), so a Llama-3-70B
        job never builds the whole model in fp32 on any rank; meta buffers
        are rebuilt as ``meta_init`` does (``buffer_init_fn``).

        ``replicate_group`` (hybrid sharding, HSDP): shards live in
        ``process_group`` (e.g. a node's xGMI group) and are replicated
        across ``replicate_group``; after the shard group's reduce-scatters
        one all-reduce of the rank's whole shard gradient sums the replicas
        (reference ATorch FSDP HYBRID_SHARD, zero_optimization.py:377-394)."""
        super().__init__()
        self.module = module
        self.pg = process_group
        init = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(process_group) if init else 1
        self.rank = dist.get_rank(process_group) if init else 0
        self.reshard = bool(reshard_after_forward) and self.world > 1
        self.rg = replicate_group
        self.replicas = dist.get_world_size(replicate_group) if (init and replicate_group is not None) else 1
        self.prefetch = bool(prefetch)
        self._sync = True
        params_all = [p for p in module.parameters()]
        if not params_all:
            raise ValueError("FlatFSDP: the module has no parameters")
        meta = any(p.is_meta for p in params_all)
        dev = params_all[0].device
        if meta:
            dev = torch.device(device) if device is not None else (
                torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
            self._materialize_buffers(module, dev, buffer_init_fn)
        dtype = params_all[0].dtype
        if any(p.dtype != dtype for p in params_all if p.requires_grad):
            raise ValueError("FlatFSDP: every trainable parameter must have one dtype (cast the model first)")
        qname: Dict[int, str] = {}
        for n, p in module.named_parameters():
            qname.setdefault(id(p), n)
        # units: the outermost wrap-class instances, then the root's leftovers
        wrap = tuple(wrap_cls or ())
        mods: List[nn.Module] = []

        def visit(m):
            for c in m.children():
                if wrap and isinstance(c, wrap):
                    mods.append(c)
                else:
                    visit(c)

        visit(module)
        seen = set()
        groups: List[Tuple[nn.Module, List[Tuple[str, nn.Parameter]], bool]] = []
        for m in mods:
            named = []
            for p in m.parameters():
                if p.requires_grad and id(p) not in seen:
                    seen.add(id(p))
                    named.append((qname[id(p)], p))
            if named:
                groups.append((m, named, False))
        root_named = [(qname[id(p)], p) for p in module.parameters() if p.requires_grad and id(p) not in seen]
        if root_named:
            groups.insert(0, (module, root_named, True))
        pad = self.world * ALIGN
        sizes = []
        for _m, named, _r in groups:
            off = sum((p.numel() + ALIGN - 1) // ALIGN * ALIGN for _n, p in named)
            sizes.append(max(pad, (off + pad - 1) // pad * pad))
        shard_total = sum(s // self.world for s in sizes)
        self._shard_data = torch.zeros(shard_total, dtype=dtype, device=dev)
        self._shard_grad = torch.zeros(shard_total, dtype=dtype, device=dev)
        masks = []
        self.units: List[_Unit] = []
        self.free_grads = self.reshard
        base = 0
        src = dist.get_global_rank(process_group, 0) if (init and process_group is not None) else 0
        for i, ((m, named, is_root), n) in enumerate(zip(groups, sizes)):
            u = _Unit(i, m, is_root)
            u.len, u.base, u.lo = n // self.world, base, self.rank * (n // self.world)
            u.shard = self._shard_data[base:base + u.len]
            u.shard_grad = self._shard_grad[base:base + u.len]
            if self.world == 1:
                u.full, u.gfull = u.shard, u.shard_grad
            else:
                u.full = torch.zeros(n, dtype=dtype, device=dev)
                u.gfull = torch.zeros(n, dtype=dtype, device=dev)
            if meta:
                named = self._rebind_meta(module, named, u.full)
            u.flat = FlatParams(None, named=named, pad_to=pad, data=u.full, grad=u.gfull, no_decay_fn=no_decay_fn,
                                lazy_zero_grad=True, device=dev)
            u.names = [nm for nm, _p in named]
            u.nbytes = n * u.full.element_size()
            if meta:
                self._init_shard(module, u, init_seed)  # gathered into ``full`` by the first forward
                u.fresh = self.world == 1
            elif self.world > 1 or self.replicas > 1:
                if sync_module_states:
                    if self.replicas > 1:  # every replica of every shard: global rank 0's values
                        dist.broadcast(u.full, src=0)
                    else:
                        dist.broadcast(u.full, src=src, group=process_group)
                with torch.no_grad():
                    u.shard.copy_(u.full[u.lo:u.lo + u.len])
                u.fresh = True
            if self.reshard and not is_root:
                # ZeRO-3: neither full-size buffer outlives the set-up of its
                # unit (the first forward gathers, the first backward takes the
                # gradient buffer): no rank ever holds two model-sized copies
                u.full.untyped_storage().resize_(0)
                u.released, u.fresh = True, False
                u.gfull.untyped_storage().resize_(0)
                u.grad_released = True
            masks.append(u.flat.decay_mask[u.lo // ALIGN:(u.lo + u.len) // ALIGN])
            self.units.append(u)
            base += u.len
        self.shard_flat = ShardFlat(self, self._shard_data, self._shard_grad, torch.cat(masks))
        self._unit_of: Dict[int, int] = {}
        for u in self.units:
            for p in u.flat.params:
                self._unit_of[id(p)] = u.idx
        self._fwd_order: Optional[List[int]] = None
        self._recording: List[int] = []
        self._expected: Optional[List[int]] = None
        self._calls = [0] * len(self.units)
        self._inflight: List[_Unit] = []  # reduce-scatters not yet known complete
        self._handles = []
        if self.world == 1 and self.replicas > 1:
            for u in self.units:
                for p in u.flat.params:
                    self._handles.append(p.register_post_accumulate_grad_hook(self._make_count_hook(u)))
        if self.world > 1:
            for u in self.units:
                if not u.is_root:
                    self._handles.append(u.module.register_forward_pre_hook(self._make_pre_forward(u)))
                    self._handles.append(u.module.register_forward_hook(self._make_post_forward(u)))
                for p in u.flat.params:
                    self._handles.append(p.register_post_accumulate_grad_hook(self._make_grad_hook(u)))
        logger.info(f"FlatFSDP: {len(self.units)} units, {shard_total} elements per rank shard "
                    f"(world {self.world}, reshard_after_forward={self.reshard})")

    # ------------------------------------------------------ meta-device init
    @staticmethod
    @torch.no_grad()
    def _materialize_buffers(module: nn.Module, dev, buffer_init_fn):
        from ..atorch.meta_init import _init_meta_buffers

        names = []
        for mname, m in module.named_modules():
            for bname, b in list(m._buffers.items()):
                if b is not None and b.is_meta:
                    m._buffers[bname] = torch.empty_like(b, device=dev)
                    names.append(f"{mname}.{bname}" if mname else bname)
                elif b is not None and b.device != dev:
                    m._buffers[bname] = b.to(dev)
        if names:
            _init_meta_buffers(module, names, dev, buffer_init_fn)

    @staticmethod
    def _rebind_meta(module: nn.Module, named, full: torch.Tensor):
        """Replace each meta parameter by a Parameter that IS its view of the
        unit buffer (FlatParams' layout: 64-element aligned, in order); a meta
        tensor cannot be re-pointed through ``.data``."""
        owners = {}
        for m in module.modules():
            for pname, p in m._parameters.items():
                if p is not None:
                    owners.setdefault(id(p), []).append((m, pname))
        out, off = [], 0
        for name, p in named:
            c = p.numel()
            if p.is_meta:
                # a fresh parameter re-pointed through .data: its own version
                # counter (a Parameter built ON the view would share the unit
                # buffer's, and every in-place gather would invalidate the
                # autograd-saved weights)
                newp = nn.Parameter(torch.empty(0, dtype=full.dtype, device=full.device), requires_grad=p.requires_grad)
                newp.data = full[off:off + c].view(p.shape)
                for m, pname in owners.get(id(p), []):
                    m._parameters[pname] = newp
                p = newp
            out.append((name, p))
            off += (c + ALIGN - 1) // ALIGN * ALIGN
        return out

    @torch.no_grad()
    def _init_shard(self, module: nn.Module, u: _Unit, seed: int):
        """This rank's element range of every parameter of ``u``: the values
        the unsharded parameter would get from ``meta_init``'s streams."""
        from ..atorch.meta_init import _fill_counter, _module_spec

        owner = {}
        for mname, m in module.named_modules():
            for pname, p in m.named_parameters(recurse=False):
                owner.setdefault(id(p), (m, pname))
        spec_fn = getattr(module, "init_spec", None)
        hi = u.lo + u.len
        for name, p, (o, c) in zip(u.names, u.flat.params, u.flat.offsets):
            a, b = max(o, u.lo), min(o + c, hi)
            if a >= b:
                continue
            m, pname = owner[id(p)]
            spec = spec_fn(name) if callable(spec_fn) else None
            if spec is None:
                spec = _module_spec(module, m, pname)
            piece = u.shard[a - u.lo:b - u.lo]
            if spec is None:
                logger.warning(f"FlatFSDP meta init: no init spec for {name} ({type(m).__name__}): zeros")
                piece.zero_()
                continue
            lo_, hi_ = (spec[1], spec[2]) if len(spec) >= 3 else (0.0, 0.0)
            _fill_counter(piece, a - o, name, seed, spec[0], lo_, hi_)

    # ------------------------------------------------------------ gathers
    def _issue_gather(self, u: _Unit):
        if self.world == 1 or u.fresh or u.work is not None:
            return
        if u.released:
            u.full.untyped_storage().resize_(u.nbytes)
            u.released = False
        u.work = dist.all_gather_into_tensor(u.full, u.shard, group=self.pg, async_op=True)

    def _ensure(self, u: _Unit):
        if self.world == 1 or u.fresh:
            return
        self._issue_gather(u)
        u.work.wait()
        u.work = None
        u.fresh = True

    def _release(self, u: _Unit):
        if not self.reshard or u.is_root or u.released or u.work is not None:
            return
        u.full.untyped_storage().resize_(0)
        u.released, u.fresh = True, False

    def _neighbour(self, u: _Unit, step: int) -> Optional[_Unit]:
        order = self._fwd_order
        if not self.prefetch or not order or u.idx not in order:
            return None
        j = order.index(u.idx) + step
        return self.units[order[j]] if 0 <= j < len(order) else None

    def _make_pre_forward(self, u: _Unit):
        def hook(_m, _args):
            if self._fwd_order is None:
                self._recording.append(u.idx)
            self._issue_gather(u)
            # (not in an activation-checkpoint recompute inside the backward:
            # the next unit in forward order has finished its backward there)
            nxt = None if _in_backward() else self._neighbour(u, +1)
            if nxt is not None:
                self._issue_gather(nxt)  # overlaps this unit's forward
            self._ensure(u)
        return hook

    def _make_post_forward(self, u: _Unit):
        def hook(_m, _args, out):
            if not torch.is_grad_enabled() or _in_backward():
                # no_grad forward, or the recompute of an activation-checkpointed
                # unit inside its backward: the parameters stay until its gradients
                return None
            self._release(u)
            if self.reshard or self.free_grads:
                ts = [t for t in _flatten(out) if torch.is_tensor(t) and t.requires_grad]
                if ts:
                    torch.autograd.graph.register_multi_grad_hook(ts, lambda _g: self._pre_backward(u), mode="any")
            return None
        return hook

    def _take_grad(self, u: _Unit):
        if not u.grad_released:
            return
        u.gfull.untyped_storage().resize_(u.nbytes)
        u.grad_released = False
        if not u.flat._fresh:  # no gradient generation open (no zero_grad since the last step): start from 0
            u.gfull.zero_()

    def _give_grad(self, u: _Unit):
        if self.free_grads and self._sync and not u.is_root and not u.grad_released:
            u.gfull.untyped_storage().resize_(0)
            u.grad_released = True

    def _drain(self, block: bool):
        """Reduce-scatters known complete (all of them with ``block``):
        their unsharded gradient buffers can be given back."""
        keep = []
        for v in self._inflight:
            if block or v.rs_work.is_completed():
                v.rs_work.wait()  # orders this stream after the collective
                v.rs_work = None
                self._give_grad(v)
            else:
                keep.append(v)
        self._inflight = keep

    def _pre_backward(self, u: _Unit):
        self._take_grad(u)
        self._issue_gather(u)
        prev = self._neighbour(u, -1)
        if prev is not None:
            self._issue_gather(prev)  # the next unit of the backward
        self._ensure(u)

    # ------------------------------------------------- gradient reduction
    def _make_grad_hook(self, u: _Unit):
        def hook(_p):
            if not self._sync:
                return
            if u.reduced:
                raise RuntimeError(f"FlatFSDP: a gradient of unit {u.idx} arrived after its reduce-scatter "
                                   "(a parameter used more often than in the first backward)")
            self._calls[u.idx] += 1
            exp = self._expected
            if exp is not None and exp[u.idx] > 0 and self._calls[u.idx] == exp[u.idx]:
                self._reduce(u)
        return hook

    def _make_count_hook(self, u: _Unit):
        def hook(_p):
            if self._sync:
                self._calls[u.idx] += 1
        return hook

    def _calls_any(self) -> bool:
        return any(self._calls)

    def _reduce(self, u: _Unit):
        self._take_grad(u)  # (a unit whose backward never ran: its gradient is zero)
        u.flat.finalize_grads()  # lazily zeroed gradients nobody wrote
        u.rs_work = dist.reduce_scatter_tensor(u.shard_grad, u.gfull, group=self.pg, async_op=True)
        u.reduced = True
        self._inflight.append(u)
        if not u.is_root:
            self._release(u)
        self._drain(block=False)

    def finish_gradient_sync(self):
        """Every unit's gradient reduced into the shard gradient (launching
        those that did not complete, e.g. units with unused parameters);
        called by the optimizer before its update."""
        for u in self.units:
            u.flat.finalize_grads()
        if not self._sync or (self.world == 1 and self.replicas == 1):
            return
        if self.world == 1:  # replicas of an unsharded model: the gradient all-reduce only
            if self._calls_any():
                dist.all_reduce(self._shard_grad, group=self.rg)
                self._calls = [0] * len(self.units)
            return
        if not any(self._calls):
            return  # no backward since the last sync
        if self._expected is None:
            self._expected = list(self._calls)
        for u in self.units:
            if not u.reduced:
                self._reduce(u)
        self._drain(block=True)
        if self.replicas > 1:  # sum the replicas' shard gradients: one collective over the shard
            dist.all_reduce(self._shard_grad, group=self.rg)
        for u in self.units:
            u.reduced = False
        self._calls = [0] * len(self.units)

    @contextmanager
    def no_sync(self):
        """Accumulate gradients locally (in the unsharded gradient buffers);
        the next synchronised backward reduces the sum."""
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def zero_grad(self):
        for u in self.units:
            if u.grad_released and not u.flat.lazy_zero:
                continue  # no storage: _take_grad zeroes it when the backward takes it again
            u.flat.zero_grad()

    # ------------------------------------------------------------- forward
    def forward(self, *args, **kwargs):
        if self.world > 1:
            if self._fwd_order is None and self._recording:
                self._fwd_order = list(self._recording)
            self._recording = []
            for u in self.units:
                if u.work is not None:  # a gather issued before the optimizer step: stale
                    u.work.wait()
                    u.work = None
                u.fresh = False  # the optimizer may have updated the shards
            for u in self.units:
                if u.is_root:
                    self._ensure(u)
        out = self.module(*args, **kwargs)
        if self.world > 1 and self._fwd_order is None:
            self._fwd_order = list(self._recording)
        return out

    # ------------------------------------------------------------ checkpoints
    def flat_shard_tensors(self) -> Tuple[Dict[str, torch.Tensor], Dict[str, dict]]:
        """This rank's element range of every flattened parameter (1-D views
        of the shard buffer) and its meta ``{"shape", "dim": -1, "offset",
        "length"}`` -- ATorch's FlatParameter shard layout."""
        return self._shard_views(self._shard_data)

    def _shard_views(self, buf: torch.Tensor) -> Tuple[Dict[str, torch.Tensor], Dict[str, dict]]:
        views, meta = {}, {}
        for u in self.units:
            hi = u.lo + u.len
            for name, p, (o, c) in zip(u.names, u.flat.params, u.flat.offsets):
                a, b = max(o, u.lo), min(o + c, hi)
                if a >= b:
                    continue
                s = u.base + (a - u.lo)
                views[name] = buf[s:s + (b - a)]
                meta[name] = {"shape": list(p.shape), "dim": -1, "offset": a - o, "length": b - a}
        return views, meta

    def full_state_dict(self) -> Dict[str, torch.Tensor]:
        """Every parameter gathered (a copy), plus the buffers."""
        out = {}
        for u in self.units:
            if self.world > 1:
                tmp = torch.empty(u.len * self.world, dtype=u.shard.dtype, device=u.shard.device)
                dist.all_gather_into_tensor(tmp, u.shard, group=self.pg)
            else:
                tmp = u.shard
            for name, p, (o, c) in zip(u.names, u.flat.params, u.flat.offsets):
                out[name] = tmp[o:o + c].view(p.shape).clone()
        for n, b in self.module.named_buffers():
            out[n] = b.detach().clone()
        return out

    def remove_hooks(self):
        for h in self._handles:
            h.remove()
        self._handles = []


def _in_backward() -> bool:
    try:
        return torch._C._current_graph_task_id() != -1
    except AttributeError:  # pragma: no cover
        return False


def _flatten(x):
    if torch.is_tensor(x):
        yield x
    elif isinstance(x, (list, tuple)):
        for v in x:
            yield from _flatten(v)
    elif isinstance(x, dict):
        for v in x.values():
            yield from _flatten(v)
