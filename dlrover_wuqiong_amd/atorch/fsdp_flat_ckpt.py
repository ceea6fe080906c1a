"""ATorch-style sharded FSDP checkpoints in safetensors, saved asynchronously
through the flash-checkpoint engine, and loaded at ANY world size.

Layout of one checkpoint directory (one file set per data-parallel rank r of
world W, suffix ``{r:05d}-{W:05d}``):

  flat_param.<suffix>    safetensors: this rank's local shard of every FSDP2
                         parameter, keyed by its fully-qualified name
  flat_meta.<suffix>     JSON: per parameter the global shape, sharded dim,
                         this rank's [offset, offset + length) along it
  optim_param.<suffix>   safetensors: "<param>-<state>" local shards of the
                         optimizer state (exp_avg, exp_avg_sq, step, ...)
  optim_meta             JSON (rank 0): param groups with parameter names
  buffers                safetensors (rank 0): model buffers
  ckpt_meta              JSON (rank 0): version, world size, wrap classes

``save_checkpoint(step, model, optimizer, path, storage_type)`` snapshots the
local shards into shared memory (the training pause) and the agent writes
the files above from shm (``FsdpFlatCheckpointSaver``, staged and moved into
place at commit; tracker ``latest_checkpointed_iteration.txt``).
``ShardTensorUtil`` reads a checkpoint lazily (memory-mapped safetensors)
and reshards it: ``load_into_model`` / ``load_optimizer`` fill a model /
optimizer sharded over a different world size, ``load_tensor_by_name``
returns full tensors (export / conversion).

FSDP2 shards every parameter on dim 0 (``torch.chunk`` semantics), so the
"flat parameter" of FSDP1 (with its alignment padding) is not needed: each
parameter's shard is stored as-is and resharding is a row-range copy.
Metadata is JSON (never unpickled).

Parity: reference atorch/atorch/utils/fsdp_async_ckpt_util.py:29-200
(FsdpCheckpointSaver, FsdpCheckpointEngine, save_checkpoint) and
fsdp_save_util.py (save_fsdp_flat_param / save_fsdp_optim_param /
ShardTensorUtil / ShardOptim).
"""

import json
import os
import struct
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..common.log import logger
from ..flash_checkpoint.checkpointer import StorageType
from ..flash_checkpoint.engine import ShardCheckpointEngine

PARAMS, BUFFERS, PARAM_META, CKPT_META, OPTIM_STATES, PARAM_GROUPS = (
    "params", "buffers", "param_meta", "ckpt_meta", "optim_states", "param_groups")
CKPT_VERSION = 2
TRACKER = "latest_checkpointed_iteration.txt"
_ST_DTYPES = {torch.bfloat16: "BF16", torch.float16: "F16", torch.float32: "F32", torch.float64: "F64",
              torch.int64: "I64", torch.int32: "I32", torch.int16: "I16", torch.int8: "I8", torch.uint8: "U8",
              torch.bool: "BOOL"}


def clean_name(name: str) -> str:
    for p in ("_fsdp_wrapped_module.", "_checkpoint_wrapped_module.", "_orig_mod.", "module."):
        name = name.replace(p, "")
    return name


# ------------------------------------------------------------- safetensors
def safetensors_dump(tensors: Dict[str, torch.Tensor], path: str):
    """Write a safetensors file streaming each tensor's bytes from where it
    lives (shm views: no copy); largest element size first, then by name."""
    items = sorted(tensors.items(), key=lambda kv: (-kv[1].element_size(), kv[0]))
    header, off = {}, 0
    for k, t in items:
        n = t.numel() * t.element_size()
        header[k] = {"dtype": _ST_DTYPES[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + n]}
        off += n
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * ((8 - len(hb) % 8) % 8)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "wb", buffering=16 << 20) as f:
        f.write(struct.pack("<Q", len(hb)))
        f.write(hb)
        for _k, t in items:
            t = t.detach()
            if t.device.type != "cpu":
                t = t.cpu()
            t = t.contiguous().reshape(-1)  # 0-dim states ("step") too
            if t.numel():
                f.write(memoryview(t.view(torch.uint8).numpy()))


# ------------------------------------------------------------- local shards
def _dp_rank_world(group=None) -> Tuple[int, int]:
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _shard_info(p) -> Tuple[torch.Tensor, dict]:
    """(local tensor, meta) of a parameter / state tensor (DTensor or plain)."""
    if hasattr(p, "_local_tensor"):
        from torch.distributed.tensor._utils import compute_local_shape_and_global_offset

        local = p._local_tensor
        shape, offset = compute_local_shape_and_global_offset(p.shape, p.device_mesh, p.placements)
        dims = [i for i, (a, b) in enumerate(zip(shape, p.shape)) if a != b]
        dim = dims[0] if dims else 0
        return local, {"shape": list(p.shape), "dim": dim, "offset": int(offset[dim]) if len(offset) else 0,
                       "length": int(shape[dim]) if len(shape) else 1}
    return p, {"shape": list(p.shape), "dim": 0, "offset": 0, "length": int(p.shape[0]) if p.dim() else 1}


def _flat_fsdp(model):
    """The ``parallel.flat_fsdp.FlatFSDP`` behind ``model`` (or None)."""
    from ..parallel.flat_fsdp import FlatFSDP

    for m in (model, getattr(model, "module", None)):
        if isinstance(m, FlatFSDP):
            return m
    return None


def get_flat_model_param(model) -> Tuple[Dict, Dict, Dict, Dict]:
    """(params {name: local shard}, buffers, param_meta, ckpt_meta)."""
    rank, world = _dp_rank_world()
    fs = _flat_fsdp(model)
    if fs is not None:
        # FlatParameter layout: this rank's element range of every flattened
        # parameter ("dim": -1), views of the live shard buffer
        views, fmeta = fs.flat_shard_tensors()
        meta = {n: dict(m, rank=rank, dtype=str(views[n].dtype).replace("torch.", "")) for n, m in fmeta.items()}
        buffers = {clean_name(k): v for k, v in fs.module.named_buffers()}
        ckpt_meta = {"version": CKPT_VERSION, "world_size": world, "layout": "flat",
                     "wrap_class": [[type(u.module).__module__, type(u.module).__name__] for u in fs.units[:2]]}
        return views, buffers, meta, ckpt_meta
    params, meta = {}, {}
    for name, p in model.named_parameters():
        local, m = _shard_info(p.detach())
        n = clean_name(name)
        params[n] = local
        meta[n] = dict(m, rank=rank, dtype=str(local.dtype).replace("torch.", ""))
    buffers = {clean_name(k): v for k, v in model.named_buffers()}
    wrap = sorted({(type(m).__module__, type(m).__name__) for m in model.modules()
                   if type(m).__name__.startswith("FSDP") and m is not model})
    ckpt_meta = {"version": CKPT_VERSION, "world_size": world, "wrap_class": [list(w) for w in wrap]}
    return params, buffers, meta, ckpt_meta


_FLAT_STATES = (("exp_avg", "exp_avg"), ("exp_avg_sq", "exp_avg_sq"), ("master_param", "master"))


def _flat_optim_views(fs, optimizer) -> Dict[str, torch.Tensor]:
    """"<param>-<state>" element-range views of a flat optimizer's state over
    a FlatFSDP shard (FusedAdamW / FusedAGD: exp_avg, exp_avg_sq, fp32
    master, one step counter)."""
    out = {}
    for key, attr in _FLAT_STATES:
        buf = getattr(optimizer, attr, None)
        if buf is None:
            continue
        views, _m = fs._shard_views(buf)
        for n, v in views.items():
            out[f"{n}-{key}"] = v
    step = getattr(optimizer, "_step_t", None)
    if step is not None:
        for n in fs.flat_shard_tensors()[0]:
            out[f"{n}-step"] = step
    return out


def get_fsdp_optim_param(model, optimizer) -> Tuple[Dict, List]:
    """(optim_states {"<param>-<state>": local tensor}, param_groups with names)."""
    fs = _flat_fsdp(model)
    if fs is not None and getattr(optimizer, "flat", None) is fs.shard_flat:
        names = [n for u in fs.units for n in u.names]
        groups = []
        for g in optimizer.param_groups:
            packed = {k: (list(v) if isinstance(v, tuple) else v) for k, v in g.items() if k != "params"}
            packed = {k: v for k, v in packed.items() if isinstance(v, (int, float, str, bool, list, type(None)))}
            packed["params"] = names
            groups.append(packed)
        return _flat_optim_views(fs, optimizer), groups
    names = {id(p): clean_name(n) for n, p in model.named_parameters()}
    groups, states = [], {}
    for g in optimizer.param_groups:
        packed = {k: (list(v) if isinstance(v, tuple) else v) for k, v in g.items() if k != "params"}
        packed = {k: v for k, v in packed.items() if isinstance(v, (int, float, str, bool, list, type(None)))}
        packed["params"] = [names[id(p)] for p in g["params"]]
        groups.append(packed)
        for p in g["params"]:
            for k, v in optimizer.state.get(p, {}).items():
                if torch.is_tensor(v):
                    local = v._local_tensor if hasattr(v, "_local_tensor") else v
                    states[f"{names[id(p)]}-{k}"] = local.detach()
    return states, groups


def _suffix(rank, world) -> str:
    return f"{rank:05d}-{world:05d}"


def ckpt_paths(path: str, rank: int, world: int) -> Dict[str, str]:
    s = _suffix(rank, world)
    return {PARAMS: f"{path}/flat_param.{s}", PARAM_META: f"{path}/flat_meta.{s}",
            OPTIM_STATES: f"{path}/optim_param.{s}", PARAM_GROUPS: f"{path}/optim_meta",
            BUFFERS: f"{path}/buffers", CKPT_META: f"{path}/ckpt_meta"}


def _write_json(obj, path):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(obj, f)


def save_fsdp_flat_param(model, path: str):
    """Synchronous write of the model files (every rank its own shard)."""
    params, buffers, meta, ckpt_meta = get_flat_model_param(model)
    rank, world = _dp_rank_world()
    p = ckpt_paths(path, rank, world)
    safetensors_dump(params, p[PARAMS])
    _write_json(meta, p[PARAM_META])
    if rank == 0:
        safetensors_dump(buffers, p[BUFFERS])
        _write_json(ckpt_meta, p[CKPT_META])


def save_fsdp_optim_param(model, optimizer, path: str):
    states, groups = get_fsdp_optim_param(model, optimizer)
    rank, world = _dp_rank_world()
    p = ckpt_paths(path, rank, world)
    safetensors_dump(states, p[OPTIM_STATES])
    if rank == 0:
        _write_json(groups, p[PARAM_GROUPS])


# ------------------------------------------------------------ flash (async)
class FsdpFlatCheckpointEngine(ShardCheckpointEngine):
    """Every rank snapshots its shards to its own shm segment; the agent
    writes the safetensors / JSON files."""

    def get_saver_class(self):
        from ..elastic_agent.ckpt_saver import FsdpFlatCheckpointSaver

        return FsdpFlatCheckpointSaver


_ENGINES: Dict[str, FsdpFlatCheckpointEngine] = {}


def _engine(checkpoint_dir, storage=None, comm_backend="") -> FsdpFlatCheckpointEngine:
    e = _ENGINES.get(checkpoint_dir)
    if e is None:
        e = _ENGINES[checkpoint_dir] = FsdpFlatCheckpointEngine(checkpoint_dir, storage, comm_backend)
    return e


def close_engines():
    for e in _ENGINES.values():
        e.close()
    _ENGINES.clear()


def _state_and_paths(model, optimizer, path, extra_sds=None, extra_paths=None):
    params, buffers, meta, ckpt_meta = get_flat_model_param(model)
    rank, world = _dp_rank_world()
    sd = {PARAMS: params, PARAM_META: meta}
    if optimizer is not None:
        states, groups = get_fsdp_optim_param(model, optimizer)
        sd[OPTIM_STATES] = states
        if rank == 0:
            sd[PARAM_GROUPS] = groups
    if rank == 0:
        sd[BUFFERS] = buffers
        sd[CKPT_META] = ckpt_meta
    paths = {k: v for k, v in ckpt_paths(path, rank, world).items() if k in sd}
    if extra_sds:
        sd.update(extra_sds)
        paths.update(extra_paths or {})
    return sd, paths


def save_checkpoint(step, model, optimizer, path, extra_sds: Optional[Dict] = None,
                    extra_paths: Optional[Dict] = None, storage_type=StorageType.DISK, comm_backend="",
                    storage=None) -> bool:
    """Flash-save one FSDP2 checkpoint in the flat safetensors layout under
    ``path`` (its parent directory holds the tracker)."""
    engine = _engine(os.path.dirname(os.path.abspath(path)), storage, comm_backend)
    sd, paths = _state_and_paths(model, optimizer, path, extra_sds, extra_paths)
    if storage_type == StorageType.MEMORY:
        return engine.save_to_memory(step, sd, paths)
    if storage_type == StorageType.DISK:
        return engine.save_to_storage(step, sd, paths)
    raise ValueError("storage_type must be StorageType.MEMORY or StorageType.DISK")


def load_checkpoint(model, optimizer, path, comm_backend="", storage=None) -> int:
    """Restore from memory in place (same world size), else from the files
    under ``path`` -- resharded to the current world size.  Returns the
    restored step from memory, -1 from storage, 0 if nothing was loaded."""
    engine = _engine(os.path.dirname(os.path.abspath(path)), storage, comm_backend)
    sd, _paths = _state_and_paths(model, optimizer, path)
    step, got = engine.get_state_dict_from_memory(target=sd)
    if step > 0 and got:
        return step
    if not os.path.exists(os.path.join(path, "ckpt_meta")):
        return 0
    util = ShardTensorUtil(path)
    util.load_into_model(model)
    if optimizer is not None:
        util.load_optimizer(model, optimizer)
    return -1


def wait_for_persist(checkpoint_dir: str, step: int, timeout: float = 600.0) -> bool:
    import time

    tracker = os.path.join(checkpoint_dir, TRACKER)
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            with open(tracker) as f:
                if f.read().strip() == str(step):
                    return True
        except OSError:
            pass
        time.sleep(0.05)
    return False


# ------------------------------------------------------------------ reading
class ShardTensorUtil:
    """Lazy reader of a flat checkpoint written at world size W; serves full
    tensors or any row range, so it loads into any world size."""

    def __init__(self, path: str):
        from safetensors import safe_open

        self.path = path
        with open(os.path.join(path, "ckpt_meta")) as f:
            self.ckpt_meta = json.load(f)
        self.world = int(self.ckpt_meta["world_size"])
        self.param_meta: Dict[str, List[dict]] = {}
        self._fds, self._ofds = {}, {}
        for r in range(self.world):
            s = _suffix(r, self.world)
            with open(os.path.join(path, f"flat_meta.{s}")) as f:
                for name, m in json.load(f).items():
                    self.param_meta.setdefault(name, []).append(dict(m, rank=r))
            self._fds[r] = safe_open(os.path.join(path, f"flat_param.{s}"), framework="pt")
            op = os.path.join(path, f"optim_param.{s}")
            if os.path.exists(op):
                self._ofds[r] = safe_open(op, framework="pt")
        for name, v in list(self.param_meta.items()):
            # hybrid sharding: replicas saved the same ranges -- keep one of each
            seen, uniq = set(), []
            for m in sorted(v, key=lambda m: (m["offset"], m["rank"])):
                key = (m["offset"], m["length"])
                if key not in seen:
                    seen.add(key)
                    uniq.append(m)
            self.param_meta[name] = uniq

    def _elements(self, fds, key_fn, name, lo: int, hi: int) -> torch.Tensor:
        """Elements [lo, hi) of the FLATTENED tensor ``name`` (1-D), whatever
        the layout it was saved in (element ranges or dim-0 row shards)."""
        metas = self.param_meta[name]
        if metas[0]["dim"] == -1:
            parts = []
            for m in metas:
                a, b = max(lo, m["offset"]), min(hi, m["offset"] + m["length"])
                if a < b:
                    parts.append(fds[m["rank"]].get_slice(key_fn(name))[a - m["offset"]:b - m["offset"]])
            if not parts:
                return torch.empty(0)
            return torch.cat(parts) if len(parts) > 1 else parts[0]
        shape = metas[0]["shape"]
        row = 1
        for d in shape[1:]:
            row *= int(d)
        r0, r1 = lo // row, (hi + row - 1) // row
        return self._rows(fds, key_fn, name, r0, r1).reshape(-1)[lo - r0 * row:hi - r0 * row]

    def _rows(self, fds, key_fn, name, lo: int, hi: int) -> torch.Tensor:
        """Rows [lo, hi) along the sharded dim of ``name`` from the shards
        that overlap them."""
        metas = self.param_meta[name]
        dim = metas[0]["dim"]
        if dim == -1:  # saved as element ranges: dim-0 rows of the full shape
            shape = list(metas[0]["shape"])
            row = 1
            for d in shape[1:]:
                row *= int(d)
            shape[0] = hi - lo
            return self._elements(fds, key_fn, name, lo * row, hi * row).view(shape)
        parts = []
        for m in metas:
            a, b = max(lo, m["offset"]), min(hi, m["offset"] + m["length"])
            if a >= b:
                continue
            fd = fds[m["rank"]]
            sl = fd.get_slice(key_fn(name))
            idx = [slice(None)] * len(m["shape"])
            idx[dim] = slice(a - m["offset"], b - m["offset"])
            parts.append(sl[tuple(idx)])
        if not parts:
            shape = list(metas[0]["shape"])
            shape[dim] = 0
            return torch.empty(shape)
        return torch.cat(parts, dim) if len(parts) > 1 else parts[0]

    def load_tensor_by_name(self, name: str) -> torch.Tensor:
        m = self.param_meta[name][0]
        if m["dim"] == -1:
            n = 1
            for d in m["shape"]:
                n *= int(d)
            return self._elements(self._fds, lambda x: x, name, 0, n).view(m["shape"])
        return self._rows(self._fds, lambda n: n, name, 0, m["shape"][m["dim"]] if m["shape"] else 1)

    def load_buffers(self) -> Dict[str, torch.Tensor]:
        from safetensors.torch import load_file

        p = os.path.join(self.path, "buffers")
        return load_file(p) if os.path.exists(p) else {}

    @staticmethod
    def _targets(t) -> Tuple[torch.Tensor, int, int, int]:
        local, m = _shard_info(t)
        return local, m["dim"], m["offset"], m["length"]

    def load_into_model(self, model):
        """Copy every parameter's rows for THIS rank's current sharding."""
        fs = _flat_fsdp(model)
        if fs is not None:
            views, meta = fs.flat_shard_tensors()
            with torch.no_grad():
                for n, v in views.items():
                    m = meta[n]
                    v.copy_(self._elements(self._fds, lambda x: x, n, m["offset"], m["offset"] + m["length"])
                            .to(v.dtype))
                bufs = self.load_buffers()
                for name, b in fs.module.named_buffers():
                    if clean_name(name) in bufs:
                        b.copy_(bufs[clean_name(name)])
            return
        with torch.no_grad():
            for name, p in model.named_parameters():
                n = clean_name(name)
                local, _dim, off, length = self._targets(p.detach())
                local.copy_(self._rows(self._fds, lambda x: x, n, off, off + length).to(local.dtype).view(local.shape))
            bufs = self.load_buffers()
            for name, b in model.named_buffers():
                if clean_name(name) in bufs:
                    b.copy_(bufs[clean_name(name)])

    def load_optimizer(self, model, optimizer):
        """Reshard the saved optimizer state into ``optimizer``'s current
        state tensors (creating them as zeros-like first if it has none)."""
        with open(os.path.join(self.path, "optim_meta")) as f:
            groups = json.load(f)
        fs = _flat_fsdp(model)
        if fs is not None and getattr(optimizer, "flat", None) is fs.shard_flat:
            for g, sg in zip(optimizer.param_groups, groups):
                for k, v in sg.items():
                    if k != "params":
                        g[k] = tuple(v) if k == "betas" else v
            _views, meta = fs.flat_shard_tensors()
            keys = {r: set(fd.keys()) for r, fd in self._ofds.items()}
            with torch.no_grad():
                for key, v in _flat_optim_views(fs, optimizer).items():
                    name, st = key.rsplit("-", 1)
                    if not any(key in ks for ks in keys.values()):
                        continue
                    if st == "step":
                        r0 = next(r for r, ks in keys.items() if key in ks)
                        v.copy_(self._ofds[r0].get_tensor(key).to(v.dtype).view(v.shape))
                        continue
                    m = meta[name]
                    v.copy_(self._elements(self._ofds, lambda x, _s=st: f"{x}-{_s}", name, m["offset"],
                                           m["offset"] + m["length"]).to(v.dtype))
            logger.info(f"flat optimizer state resharded from world {self.world} checkpoint {self.path}")
            return
        names = {clean_name(n): p for n, p in model.named_parameters()}
        for g, sg in zip(optimizer.param_groups, groups):
            for k, v in sg.items():
                if k != "params":
                    g[k] = tuple(v) if k == "betas" else v
        keys = {r: set(fd.keys()) for r, fd in self._ofds.items()}
        all_keys = set().union(*keys.values()) if keys else set()
        with torch.no_grad():
            for name, p in names.items():
                st = optimizer.state.get(p)
                if not st:
                    # a fresh optimizer: create the saved states for this rank's rows
                    st = optimizer.state[p] = {}
                    plocal, _d, off, length = self._targets(p.detach())
                    for key in sorted(k for k in all_keys if k.startswith(name + "-")):
                        k = key[len(name) + 1:]
                        r0 = next(r for r, ks in keys.items() if key in ks)
                        if len(self._ofds[r0].get_slice(key).get_shape()) == 0:  # scalar state ("step")
                            v = self._ofds[r0].get_tensor(key)
                        else:
                            v = self._rows(self._ofds, lambda x, _k=k: f"{x}-{_k}", name, off, off + length)
                            v = v.to(plocal.device).view(plocal.shape)
                            if hasattr(p, "device_mesh"):
                                from torch.distributed.tensor import DTensor

                                v = DTensor.from_local(v, p.device_mesh, p.placements, run_check=False,
                                                       shape=p.shape, stride=p.stride())
                        st[k] = v
                    continue
                for k, v in st.items():
                    key = f"{name}-{k}"
                    if not any(key in ks for ks in keys.values()):
                        continue
                    if not torch.is_tensor(v):
                        continue
                    local, _dim, off, length = self._targets(v)
                    if local.dim() == 0 or local.shape != _shard_info(p.detach())[0].shape:
                        # scalar / unsharded state ("step"): any rank's copy
                        r0 = next(r for r, ks in keys.items() if key in ks)
                        local.copy_(self._ofds[r0].get_tensor(key).to(local.dtype).view(local.shape))
                        continue
                    rows = self._rows(self._ofds, lambda x, _k=k: f"{x}-{_k}", name, off, off + length)
                    local.copy_(rows.to(local.dtype).view(local.shape))
        logger.info(f"optimizer state resharded from world {self.world} checkpoint {self.path}")
