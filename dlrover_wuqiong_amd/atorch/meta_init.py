"""Meta-device model initialisation for FSDP2 and ``sync_module_states``.

A model built under ``init_empty_weights()`` (accelerate) or
``torch.device("meta")`` holds no parameter memory.  ``auto_accelerate``'s
``fsdp`` strategy shards it first (``fully_shard`` on meta parameters), then
materialises ONLY this rank's shards on the device (``to_empty``) and fills
them, so a Llama-3-70B job never builds the whole model on any rank:

* ``init_from``: a safetensors file / directory (a HF checkpoint): every
  rank reads only its rows of every parameter (``safe_open.get_slice``);
* ``param_init_fn``: a user callable applied to every module (FSDP1
  ``param_init_fn`` semantics), on the sharded parameters;
* default: :func:`deterministic_init_` -- each parameter is filled from a
  counter-based stream (one seeded generator per 2^20-element block of the
  FULL tensor, keyed by the parameter name), so a shard gets exactly the
  values the same parameter would have unsharded, for any world size or
  mesh.  The distribution per parameter comes from the model's
  ``init_spec(name)`` when it has one (this package's GPT-2 / Llama),
  else from the module type (Linear / Embedding: normal(0,
  ``config.initializer_range`` or 0.02); norms: ones; biases: zeros).

``sync_module_states=True``: rank 0's initial weights win.  A fully built
model is broadcast from rank 0 before sharding; when only rank 0 holds a
real model and the others are meta (the reference's "rank 0 loads the
checkpoint" pattern), rank 0's full tensors are scattered shard by shard
(``distribute_tensor(..., src_data_rank=0)``).

Reference: ``atorch/auto/opt_lib/zero_optimization.py:328-369`` (meta model,
``param_init_fn`` / per-shard flat-param loading, ``sync_module_states``)
and ``atorch/utils/fsdp_init_util.py:24-364``.
"""

import os
import zlib
from typing import Callable, Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..common.log import logger

BLOCK = 1 << 20  # elements per seeded block of the full tensor


def is_meta(model: nn.Module) -> bool:
    for p in model.parameters():
        loc = p.to_local() if hasattr(p, "to_local") else p
        if loc.is_meta:
            return True
    return False


def _local(p):
    return p.to_local() if hasattr(p, "to_local") else p


def _global_offset(p) -> int:
    """Flat element offset of this rank's (row-contiguous) local piece in the
    full tensor (0 for a plain tensor)."""
    if not hasattr(p, "to_local"):
        return 0
    from torch.distributed.tensor._utils import compute_local_shape_and_global_offset

    _shape, off = compute_local_shape_and_global_offset(p.shape, p.device_mesh, p.placements)
    strides = torch.empty(p.shape, device="meta").stride()
    return sum(o * s for o, s in zip(off, strides))


def _block_seed(seed: int, key: int, j: int) -> int:
    return ((seed * 1000003 + key) * 1000003 + j) % (1 << 63)


@torch.no_grad()
def _fill_counter(local: torch.Tensor, off: int, name: str, seed: int, kind: str, a: float, b: float):
    """Fill ``local`` (row-contiguous piece of the full tensor starting at
    flat element ``off``) with the values of the full tensor's blocks."""
    flat = local.view(-1)
    n = flat.numel()
    if kind == "zeros":
        flat.zero_()
        return
    if kind == "ones":
        flat.fill_(1.0)
        return
    key = zlib.crc32(name.encode())
    dev = local.device
    j0, j1 = off // BLOCK, (off + n + BLOCK - 1) // BLOCK
    for j in range(j0, j1):
        lo, hi = max(off, j * BLOCK), min(off + n, (j + 1) * BLOCK)
        g = torch.Generator(device=dev).manual_seed(_block_seed(seed, key, j))
        blk = torch.empty(BLOCK, dtype=torch.float32, device=dev)
        if kind == "normal":
            blk.normal_(a, b, generator=g)
        else:  # uniform
            blk.uniform_(a, b, generator=g)
        flat[lo - off: hi - off].copy_(blk[lo - j * BLOCK: hi - j * BLOCK])


def _module_spec(model, module: nn.Module, pname: str):
    std = float(getattr(getattr(model, "config", None), "initializer_range", 0.02) or 0.02)
    cls = type(module).__name__
    if pname == "bias":
        return ("zeros",)
    if isinstance(module, (nn.Linear, nn.Embedding)) or cls in ("ColumnParallelLinear", "RowParallelLinear",
                                                                 "VocabParallelEmbedding"):
        return ("normal", 0.0, std)
    if "Norm" in cls and pname == "weight":
        return ("ones",)
    return None


@torch.no_grad()
def deterministic_init_(model: nn.Module, seed: int = 0) -> Dict[str, int]:
    """Initialise every parameter (plain or DTensor-sharded) with values that
    do not depend on how it is sharded.  Returns counts per init kind."""
    spec_fn = getattr(model, "init_spec", None)
    counts: Dict[str, int] = {}
    for mname, module in model.named_modules():
        for pname, p in module.named_parameters(recurse=False):
            full = f"{mname}.{pname}" if mname else pname
            spec = spec_fn(full) if callable(spec_fn) else None
            if spec is None:
                spec = _module_spec(model, module, pname)
            local = _local(p)
            if spec is None:
                if hasattr(module, "reset_parameters"):
                    module.reset_parameters()  # sharding-dependent values: logged
                    kind = "reset_parameters"
                else:
                    local.zero_()
                    kind = "zeros(unknown)"
                logger.warning(f"meta init: no init spec for {full} ({type(module).__name__}): {kind}")
            else:
                kind = spec[0]
                a, b = (spec[1], spec[2]) if len(spec) >= 3 else (0.0, 0.0)
                if local.numel():
                    _fill_counter(local, _global_offset(p), full, seed, kind, a, b)
            counts[kind] = counts.get(kind, 0) + 1
    return counts


@torch.no_grad()
def load_shards_from_safetensors(model: nn.Module, path: str, prefix: str = "") -> int:
    """Read only this rank's rows of every parameter from a safetensors file
    (or a directory of them).  Returns the number of parameters loaded."""
    from safetensors import safe_open

    files = [path] if os.path.isfile(path) else sorted(
        os.path.join(path, f) for f in os.listdir(path) if f.endswith(".safetensors"))
    where = {}
    for f in files:
        with safe_open(f, framework="pt") as h:
            for k in h.keys():
                where[k] = f
    n = 0
    handles = {}
    try:
        for name, p in model.named_parameters():
            key = prefix + name
            if key not in where:
                raise KeyError(f"{key} not in {path}")
            h = handles.get(where[key])
            if h is None:
                h = handles[where[key]] = safe_open(where[key], framework="pt").__enter__()
            local = _local(p)
            if hasattr(p, "to_local"):
                from torch.distributed.tensor._utils import compute_local_shape_and_global_offset

                shape, off = compute_local_shape_and_global_offset(p.shape, p.device_mesh, p.placements)
                sl = h.get_slice(key)
                idx = tuple(slice(o, o + s) for o, s in zip(off, shape))
                src = sl[idx] if local.numel() else None
            else:
                src = h.get_tensor(key)
            if src is not None:
                local.copy_(src.to(local.dtype))
            n += 1
    finally:
        for h in handles.values():
            h.__exit__(None, None, None)
    return n


def _bucketed_broadcast(tensors, src: int, group=None, bucket_bytes: int = 256 << 20):
    from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

    by_dev = {}
    for t in tensors:
        by_dev.setdefault((t.device, t.dtype), []).append(t)
    for ts in by_dev.values():
        cur, size = [], 0
        for t in ts + [None]:
            if t is not None:
                cur.append(t)
                size += t.numel() * t.element_size()
            if cur and (t is None or size >= bucket_bytes):
                flat = _flatten_dense_tensors([c.data for c in cur])
                dist.broadcast(flat, src=src, group=group)
                for c, v in zip(cur, _unflatten_dense_tensors(flat, [c.data for c in cur])):
                    c.data.copy_(v)
                cur, size = [], 0


@torch.no_grad()
def sync_full_module_states(model: nn.Module, src: int = 0, group=None):
    """Broadcast a fully built (unsharded) model's parameters and buffers
    from global rank ``src`` (before sharding)."""
    _bucketed_broadcast([p for p in model.parameters()] + [b for b in model.buffers()], src, group)


def capture_full_states(model: nn.Module) -> Optional[Dict[str, torch.Tensor]]:
    """On a rank with a real model: name -> full tensor (kept alive across
    ``fully_shard`` for the scatter of :func:`scatter_from_rank0`)."""
    if is_meta(model):
        return None
    return {n: p.detach() for n, p in model.named_parameters()}


@torch.no_grad()
def scatter_from_rank0(model: nn.Module, full: Optional[Dict[str, torch.Tensor]], device):
    """Every rank's local shards from global rank 0's full tensors."""
    from torch.distributed.tensor import distribute_tensor

    me = dist.get_rank()
    for name, p in model.named_parameters():
        if hasattr(p, "to_local"):
            if me == 0:
                src = full[name].to(device=device, dtype=p.dtype)
            else:
                src = torch.empty(p.shape, dtype=p.dtype, device=device)
            d = distribute_tensor(src, p.device_mesh, p.placements, src_data_rank=0)
            _local(p).copy_(d.to_local())
            del src, d
        else:
            t = full[name].to(device=device, dtype=p.dtype) if me == 0 else p.data
            dist.broadcast(t, src=0)
            p.data.copy_(t)


def _init_meta_buffers(model: nn.Module, names, device, buffer_init_fn: Optional[Callable] = None):
    """Buffers created under ``torch.device("meta")`` hold no values after
    ``to_empty``.  Recompute them: ``buffer_init_fn(module)`` if given, else
    a parameter-free module that carries its ``config`` (HF rotary
    embeddings: ``inv_freq`` / ``original_inv_freq``) is rebuilt on the CPU
    from that config and its buffers copied.  Anything else fails loudly --
    training on uninitialised buffers is silent garbage."""
    owners = {}
    for n in names:
        mod_name, _, buf = n.rpartition(".")
        owners.setdefault(mod_name, []).append(buf)
    unresolved = []
    for mod_name, bufs in owners.items():
        m = model.get_submodule(mod_name) if mod_name else model
        if buffer_init_fn is not None:
            buffer_init_fn(m)
            continue
        fresh = None
        if getattr(m, "config", None) is not None and not list(m.parameters(recurse=False)):
            try:
                with torch.device("cpu"):
                    fresh = type(m)(m.config)
            except Exception:
                fresh = None
        if fresh is None:
            unresolved += [f"{mod_name}.{b}" if mod_name else b for b in bufs]
            continue
        for b in bufs:
            getattr(m, b).copy_(getattr(fresh, b).to(device))
        for k, v in vars(fresh).items():  # derived scalars set next to the buffers (attention_scaling, ...)
            if not k.startswith("_") and isinstance(v, (int, float)) and not isinstance(v, bool):
                setattr(m, k, v)
    if unresolved:
        raise RuntimeError(f"buffers created on the meta device have no initialiser: {unresolved[:8]} "
                           f"({len(unresolved)} total); pass buffer_init_fn or build them on a real device")


@torch.no_grad()
def materialize_sharded(model: nn.Module, device, cfg: Optional[dict] = None,
                        full_rank0: Optional[Dict[str, torch.Tensor]] = None) -> str:
    """After ``fully_shard`` on a (partly) meta model: allocate this rank's
    shards on ``device`` and fill them.  Returns the method used."""
    cfg = cfg or {}
    saved_buffers = {n: b.detach().clone() for n, b in model.named_buffers() if not b.is_meta}
    meta_buffers = [n for n, b in model.named_buffers() if b.is_meta]
    rank0_real = bool(cfg.get("sync_module_states") and cfg.get("_rank0_real"))
    model.to_empty(device=device)
    for n, b in model.named_buffers():
        if n in saved_buffers:
            b.copy_(saved_buffers[n])
    if rank0_real:
        # rank 0 built the real model: its buffers (rotary inv_freq, ...) are
        # the truth; the other ranks' were created on meta and are garbage
        # (reference atorch/utils/fsdp_init_util.py:340
        # _sync_module_params_and_buffers)
        for _n, b in model.named_buffers():
            dist.broadcast(b.data, src=0)  # on `device` after to_empty
    elif meta_buffers:
        _init_meta_buffers(model, meta_buffers, device, cfg.get("buffer_init_fn"))
    init_fn: Optional[Callable] = cfg.get("param_init_fn")
    if rank0_real:
        scatter_from_rank0(model, full_rank0, device)
        how = "scatter_from_rank0"
    elif cfg.get("init_from"):
        load_shards_from_safetensors(model, cfg["init_from"], cfg.get("init_from_prefix", ""))
        how = "safetensors_shards"
    elif init_fn is not None:
        for m in model.modules():
            init_fn(m)
        how = "param_init_fn"
    else:
        deterministic_init_(model, seed=int(cfg.get("init_seed", 0)))
        how = "deterministic"
    return how
