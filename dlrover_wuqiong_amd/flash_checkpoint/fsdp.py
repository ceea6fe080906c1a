"""Flash checkpoint for FSDP / DTensor-sharded training; DCP-compatible on disk.

Parity: reference ``dlrover/trainer/torch/flash_checkpoint/fsdp.py``
(``FsdpShardCheckpointer`` :36-150, ``FsdpFullCheckpointer`` :152-290) and
``fsdp_engine.py`` (``SharedMemoryWriter`` :158, ``SharedMemoryReader`` :224,
``FsdpCheckpointEngine`` :416-560).

How it differs from the reference (and why it is faster on MI355X):

* The reference runs a full ``dist_cp.save`` on every save with a storage
  writer that ``torch.save``-serialises every item into shared memory on the
  CPU: a planning collective plus a CPU serialisation pass inside the
  training loop.  Here the DCP *plan* (local write items + global
  ``Metadata``) is computed once per state-dict layout (one collective on the
  gloo control group, re-run only when the layout changes) and cached.  A
  save is then exactly the engine's device snapshot of the local shard
  tensors -- one multi-copy kernel into HBM staging plus an async D2H flush --
  the same cost as a DDP snapshot of the same bytes.
* The agent turns the raw shard into the standard DCP layout: one
  ``__{rank}_0.distcp`` per rank holding one ``torch.save`` blob per write
  item (byte items verbatim) and, at commit on node 0, ``.metadata`` built
  from the cached global plan plus every rank's storage index.  A plain
  ``torch.distributed.checkpoint.load`` with ``FileSystemReader`` reads it,
  including at a different world size (resharding).
* Memory restore with an unchanged plan copies straight into the live local
  shards (pipelined pin + H2D), byte items come back via
  ``torch.load(weights_only=True)``, then ``set_state_dict``.
"""

import io
import json
import os
import pickle
import time
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..common.constants import CheckpointConstant
from ..common.log import logger
from ..common.serialize import restricted_loads, safe_torch_load
from ..common.storage import CheckpointStorage, PosixDiskStorage, get_checkpoint_storage
from .checkpointer import Checkpointer, StorageType
from .engine import FullCheckpointEngine, ShardCheckpointEngine, check_all_rank_ready

DCP_KEY = "dcp"
PARTS_DIR = ".dwamd_dcp_parts"
META_PART = "metadata.pkl"


def _dcp():
    from torch.distributed.checkpoint.default_planner import DefaultSavePlanner
    from torch.distributed.checkpoint.metadata import MetadataIndex
    from torch.distributed.checkpoint.planner import WriteItemType

    return DefaultSavePlanner, MetadataIndex, WriteItemType


def _item_sig(it) -> Tuple:
    td = it.tensor_data
    off = tuple(it.index.offset) if it.index.offset is not None else None
    if td is None:
        return (it.index.fqn, off, it.index.index, int(it.type.value))
    return (it.index.fqn, off, it.index.index, int(it.type.value), tuple(td.size), tuple(td.chunk.sizes),
            str(td.properties.dtype))


def _leaf_sig(v) -> Tuple:
    """What fixes a flattened state-dict leaf's write items: global shape,
    dtype, placements and local shard shape of a DTensor; shape and dtype of
    a plain tensor; only the type of a byte item (its value is re-serialised
    every save).  Other tensor subclasses (ShardedTensor) never match."""
    from torch.distributed.tensor import DTensor

    if isinstance(v, DTensor):
        return ("D", tuple(v.shape), str(v.dtype), tuple(str(p) for p in v.placements),
                tuple(v._local_tensor.shape), id(v.device_mesh))
    if type(v) is torch.Tensor or type(v) is torch.nn.Parameter:
        return ("T", tuple(v.shape), str(v.dtype))
    if torch.is_tensor(v):
        return ("X", id(object()))
    return ("O", type(v).__name__)


class _DcpPlan:
    """Cached result of DCP planning for one state-dict layout."""

    def __init__(self, sig, items, persist: List[bool], metadata_bytes: Optional[bytes]):
        self.sig = sig
        self.items = items
        self.persist = persist
        self.metadata_bytes = metadata_bytes


class DcpPlanner:
    """Plans (and caches) which local items a rank writes and the global
    DCP metadata, using torch's ``DefaultSavePlanner`` so the on-disk
    format is exactly what ``dist_cp.load`` expects."""

    def __init__(self, ctl_group=None):
        self._ctl_group = ctl_group
        self._plan: Optional[_DcpPlan] = None
        self._leaves: Optional[Tuple] = None  # leaf signatures the cached plan was made from
        self.fast_hits = 0

    def setup(self, state_dict: Dict[str, Any]):
        DefaultSavePlanner, _, _ = _dcp()
        rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        planner = DefaultSavePlanner()
        planner.set_up_planner(state_dict, storage_meta=None, is_coordinator=(rank == 0))
        # the local plan is a function of the flattened leaves' layout: when
        # that is unchanged, skip create_local_plan (per-DTensor offset math,
        # ~0.1 ms a leaf, tens of ms for a few thousand) and reuse the items
        leaves = tuple((k, _leaf_sig(v)) for k, v in planner.state_dict.items())
        local = None
        hit = self._plan is not None and self._leaves == leaves
        if not hit:
            local = planner.create_local_plan()
            sig = tuple(_item_sig(it) for it in local.items)
            hit = self._plan is not None and self._plan.sig == sig
        distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        if distributed:
            hit = check_all_rank_ready(self._ctl_group, hit)
        if hit:
            self._leaves = leaves
            self.fast_hits += int(local is None)
        else:
            if local is None:  # another rank's layout changed: plan afresh everywhere
                local = planner.create_local_plan()
                sig = tuple(_item_sig(it) for it in local.items)
            self._leaves = leaves
            if distributed:
                plans = [None] * dist.get_world_size()
                dist.all_gather_object(plans, local, group=self._ctl_group)
            else:
                plans = [local]
            # deterministic: every rank derives the same global plan, no scatter
            global_plans, metadata = planner.create_global_plan(plans)
            mine = {(it.index.fqn, tuple(it.index.offset) if it.index.offset is not None else None)
                    for it in global_plans[rank].items}
            persist = [(it.index.fqn, tuple(it.index.offset) if it.index.offset is not None else None) in mine
                       for it in local.items]
            metadata.storage_data = {}
            md_bytes = pickle.dumps(metadata) if rank == 0 else None
            self._plan = _DcpPlan(sig, list(local.items), persist, md_bytes)
        return planner, self._plan


def build_dcp_payload(planner, plan: _DcpPlan, rank: int) -> Dict[str, Any]:
    """The flat state dict handed to the flash engine: the local write items'
    tensors (views of the live shards) plus byte items as Python bytes."""
    _, _, WriteItemType = _dcp()
    tensors: Dict[str, Any] = {}
    index = []
    views: Dict[str, torch.Tensor] = {}
    for n, it in enumerate(plan.items):
        data = planner.resolve_data(it)
        key = str(n)
        if it.type == WriteItemType.BYTE_IO:
            tensors[key] = bytes(data.getbuffer())
        else:
            t = data.detach()
            if t.is_contiguous():
                tensors[key] = t
            else:
                # snapshot from a contiguous copy; a restore lands in the copy
                # and is written back through the live view (restore_views)
                tensors[key] = t.contiguous()
                views[key] = t
        off = list(it.index.offset) if it.index.offset is not None else None
        index.append([it.index.fqn, off, it.index.index, int(it.type.value), bool(plan.persist[n])])
    return {"items": tensors, "index": index, "rank": rank, "metadata": plan.metadata_bytes, "_views": views}


def restore_views(payload: Dict[str, Any], views: Dict[str, torch.Tensor]):
    """Copy restored contiguous stand-ins back into their non-contiguous live
    tensors (``views`` = the ``_views`` entry popped off the payload)."""
    with torch.no_grad():
        for key, live in views.items():
            live.copy_(payload["items"][key])


# ---------------------------------------------------------------- persisting
def _open_writer(storage: CheckpointStorage, path: str):
    if isinstance(storage, PosixDiskStorage):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        return open(path, "wb", buffering=16 << 20), True
    return io.BytesIO(), False


def persist_dcp_shard(storage: CheckpointStorage, sd: Dict[str, Any], cfg) -> str:
    """Agent side: write one rank's shard as ``__{rank}_0.distcp`` plus its
    storage index part (and rank 0's pickled global metadata)."""
    payload = sd[DCP_KEY]
    path = cfg.paths[DCP_KEY]
    rank = int(payload["rank"])
    rel = f"__{rank}_0.distcp"
    fpath = os.path.join(path, rel)
    entries = []
    f, is_file = _open_writer(storage, fpath)
    try:
        for n, (fqn, off, idx, _typ, persist) in enumerate(payload["index"]):
            if not persist:
                continue
            data = payload["items"][str(n)]
            start = f.tell()
            if isinstance(data, (bytes, bytearray)):
                f.write(data)
            else:
                torch.save(data, f)
            entries.append([fqn, off, idx, rel, start, f.tell() - start])
        if is_file:
            f.flush()
            os.fsync(f.fileno())
        else:
            storage.write(f.getvalue(), fpath)
    finally:
        f.close()
    parts = os.path.join(path, PARTS_DIR)
    storage.write(json.dumps(entries), os.path.join(parts, f"{rank}.json"))
    if payload.get("metadata"):
        storage.write(payload["metadata"], os.path.join(parts, META_PART))
    return path


def finalize_dcp_checkpoint(storage: CheckpointStorage, path: str, world_size: int) -> bool:
    """Node 0 at commit: merge every rank's storage index into the cached
    global metadata and write ``.metadata`` (torch DCP format)."""
    from torch.distributed.checkpoint.filesystem import _StorageInfo

    _, MetadataIndex, _ = _dcp()
    parts = os.path.join(path, PARTS_DIR)
    if not storage.exists(os.path.join(parts, META_PART)):
        logger.error(f"DCP metadata part missing under {parts}")
        return False
    names = [n for n in storage.listdir(parts) if n.endswith(".json")]
    if len(names) < world_size:
        logger.error(f"DCP storage index incomplete: {len(names)}/{world_size} ranks")
        return False
    md = restricted_loads(storage.read(os.path.join(parts, META_PART), mode="rb"))  # rank 0 of this job
    storage_data = {}
    for name in names:
        for fqn, off, idx, rel, start, length in json.loads(storage.read(os.path.join(parts, name))):
            key = MetadataIndex(fqn, torch.Size(off) if off is not None else None, idx)
            storage_data[key] = _StorageInfo(rel, start, length)
    md.storage_data = storage_data
    storage.write(pickle.dumps(md), os.path.join(path, ".metadata"))
    storage.safe_rmtree(parts)
    return True


# ------------------------------------------------------------------ engine
class FsdpCheckpointEngine(ShardCheckpointEngine):
    """Shard engine whose payload is a DCP write plan's local items."""

    def __init__(self, checkpoint_dir, storage=None, comm_backend="",
                 save_timeout=CheckpointConstant.SAVE_TIMEOUT, replica_count=0):
        super().__init__(checkpoint_dir, storage, comm_backend=comm_backend, save_timeout=save_timeout,
                         replica_count=replica_count)
        self._planner = DcpPlanner(self._ctl_group)

    def get_saver_class(self):
        from ..elastic_agent.ckpt_saver import FsdpDcpSaver

        return FsdpDcpSaver

    def _payload(self, state_dict):
        planner, plan = self._planner.setup(state_dict)
        return planner, plan, build_dcp_payload(planner, plan, self._rank)

    def save_to_memory(self, step, state_dict, paths):
        _, _, payload = self._payload(state_dict)
        payload.pop("_views", None)
        return super().save_to_memory(step, {DCP_KEY: payload}, paths)

    def save_to_storage(self, step, state_dict, paths):
        ok = True
        if step > self._cached_step:
            self._storage_save = True  # a requested persist waits for a busy staging buffer
            try:
                ok = self.save_to_memory(step, state_dict, paths)
            finally:
                self._storage_save = False
        if dist.is_available() and dist.is_initialized():
            dist.barrier(group=self._ctl_group)
        if ok:
            self._notify_persist(step)
        return ok

    def load_into(self, state_dict: Dict[str, Any], resume_path: str = "") -> int:
        """Fill ``state_dict`` (DTensor / ShardedTensor / tensor / object
        leaves) in place.  Returns the restored step (-1 if the storage
        checkpoint has no step information), 0 if nothing was restored."""
        step = self._load_from_memory(state_dict)
        if step > 0:
            return step
        return self._load_from_storage_dcp(state_dict, resume_path)

    def _load_from_memory(self, state_dict) -> int:
        from torch.distributed.checkpoint._traverse import set_element

        planner, plan, payload = self._payload(state_dict)
        views = payload.pop("_views", {})
        # same tree as the saved one -> tensors restored in place into the live shards
        step, sd = self.get_state_dict_from_memory(target={DCP_KEY: payload})
        if step <= 0 or not sd:
            return 0
        saved = sd[DCP_KEY]
        if [x[:4] for x in saved["index"]] != [x[:4] for x in payload["index"]]:
            logger.info("in-memory DCP plan differs from the current one; loading from storage")
            return 0
        items = saved["items"]
        for n, (fqn, _off, _idx, _typ, _p) in enumerate(saved["index"]):
            v = items[str(n)]
            if isinstance(v, (bytes, bytearray)):
                obj = safe_torch_load(io.BytesIO(v))
                set_element(state_dict, planner.mappings[fqn], obj)
            elif torch.is_tensor(v):
                dst = payload["items"][str(n)]
                if v.data_ptr() != dst.data_ptr():
                    with torch.no_grad():
                        dst.copy_(v.view(dst.shape))
        restore_views(payload, views)
        return step

    def _resume_dir(self, resume_path: str) -> str:
        if resume_path:
            return resume_path
        tracker = os.path.join(self.checkpoint_dir, CheckpointConstant.TRACER_FILE_NAME)
        content = self.storage.read(tracker)
        return os.path.join(self.checkpoint_dir, str(content).strip()) if content else ""

    def _load_from_storage_dcp(self, state_dict, resume_path="") -> int:
        import torch.distributed.checkpoint as dist_cp

        path = self._resume_dir(resume_path)
        ok = bool(path) and os.path.exists(os.path.join(path, ".metadata"))
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            ok = check_all_rank_ready(self._ctl_group, ok)
        if not ok:
            return 0
        t0 = time.perf_counter()
        plan = self._fast_storage_plan(state_dict, path) if os.environ.get("DWAMD_FAST_STORAGE_LOAD", "1") == "1" \
            else None
        fast = plan is not None
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            fast = check_all_rank_ready(self._ctl_group, fast)  # all ranks take the same path
        if fast:
            self._run_fast_storage_plan(state_dict, plan)
            self.last_restore_source = "storage"
        else:
            dist_cp.load(state_dict, storage_reader=dist_cp.FileSystemReader(path),
                         process_group=self._ctl_group if dist.is_initialized() else None)
            self.last_restore_source = "storage(dcp)"
        self.last_storage_load_stats = dict(getattr(self, "_fast_stats", {}) if fast else {},
                                            sec=round(time.perf_counter() - t0, 4), fast=fast)
        base = os.path.basename(os.path.normpath(path))
        return int(base) if base.isdigit() else -1

    def _fast_storage_plan(self, state_dict, path):
        """Same DCP layout as this rank's current shards (same world size and
        sharding): map every local item to its byte range in the ``.distcp``
        files -- None when any item is missing or differs (resharding: the
        stock DCP reader handles it)."""
        from torch.distributed.checkpoint.metadata import Metadata

        from .storage_loader import TorchArchive, _pair, _regions

        try:
            with open(os.path.join(path, ".metadata"), "rb") as f:
                md = restricted_loads(f.read())
            if not isinstance(md, Metadata):
                return None
            lookup = {(k.fqn, tuple(k.offset) if k.offset is not None else None): v
                      for k, v in md.storage_data.items()}
            planner, _plan, payload = self._payload(state_dict)
            views = payload.pop("_views", {})
            by_file: Dict[str, list] = {}
            byte_items = []
            for n, (fqn, off, _idx, _typ, _p) in enumerate(payload["index"]):
                info = lookup.get((fqn, tuple(off) if off is not None else None))
                if info is None:
                    return None
                fpath = os.path.join(path, info.relative_path)
                v = payload["items"][str(n)]
                if isinstance(v, (bytes, bytearray)):
                    byte_items.append((fqn, fpath, info.offset, info.length))
                    continue
                arc = TorchArchive(fpath, info.offset, info.length)
                pairs = []
                _pair(arc.tree, v, pairs)
                regs, slow = _regions(pairs, arc)
                if slow:
                    return None
                by_file.setdefault(fpath, []).extend(regs)
            return planner, payload, views, by_file, byte_items
        except (OSError, KeyError, ValueError, EOFError, pickle.UnpicklingError) as e:
            logger.info(f"fast DCP restore not applicable ({type(e).__name__}: {e}); using dist_cp.load")
            return None

    def _run_fast_storage_plan(self, state_dict, plan):
        """Parallel O_DIRECT reads of this rank's ``.distcp`` ranges straight
        into the live shards (pinned bounce buffers, pipelined H2D)."""
        from torch.distributed.checkpoint._traverse import set_element

        from .storage_loader import _Reader, stream_regions_into

        planner, payload, views, by_file, byte_items = plan
        direct = os.environ.get("DWAMD_STORAGE_DIRECT", "1") == "1"
        nb = 0
        for fpath, regs in by_file.items():
            nb += stream_regions_into(_Reader(fpath, direct, False, 16), os.path.getsize(fpath), regs)
        for fqn, fpath, off, length in byte_items:
            with open(fpath, "rb") as f:
                f.seek(off)
                obj = safe_torch_load(io.BytesIO(f.read(length)))
            set_element(state_dict, planner.mappings[fqn], obj)
        restore_views(payload, views)
        self._fast_stats = {"bytes_read": nb, "files": len(by_file)}


# ------------------------------------------------------------ checkpointers
_SD_INFO: Dict[Tuple, Any] = {}  # (model, optimizer, full) ids -> torch's _StateDictInfo


def _model_optim_state(model, optimizer, full: bool):
    from torch.distributed.checkpoint.state_dict import StateDictOptions, get_state_dict

    opts = StateDictOptions(full_state_dict=full, cpu_offload=False)
    if optimizer is None:
        from torch.distributed.checkpoint.state_dict import get_model_state_dict

        return get_model_state_dict(model, options=opts), None
    try:
        # torch's get_state_dict re-derives the FQN / parameter maps of the
        # model on every call (_verify_options, ~20 ms for a 1.5 B model):
        # they are fixed for a given model + optimizer, so keep them
        from torch.distributed.checkpoint import state_dict as _tsd

        key = (id(model), id(optimizer), full, len(optimizer.param_groups))
        info = _SD_INFO.get(key)
        if info is None:
            info = _tsd._verify_options(model, (optimizer,), optim_only=False, options=opts)
            _SD_INFO.clear()
            _SD_INFO[key] = info
        with _tsd._gc_context():
            msd = _tsd._get_model_state_dict(model, info)
            osd = _tsd._get_optim_state_dict(model, (optimizer,), info)
        return msd, osd
    except (AttributeError, TypeError):  # private API moved: the public call
        return get_state_dict(model, optimizer, options=opts)


def _set_model_optim_state(model, optimizer, msd, osd, full: bool):
    from torch.distributed.checkpoint.state_dict import StateDictOptions, set_model_state_dict, set_state_dict

    opts = StateDictOptions(full_state_dict=full, strict=True)
    if optimizer is None or osd is None:
        set_model_state_dict(model, msd, options=opts)
    else:
        set_state_dict(model, optimizer, model_state_dict=msd, optim_state_dict=osd, options=opts)


class FsdpShardCheckpointer(Checkpointer):
    """Sharded (FSDP1 ``SHARDED_STATE_DICT`` / FSDP2 DTensor / any DTensor
    model) flash checkpointer.

    >>> ckpt = FsdpShardCheckpointer("/ckpt")
    >>> ckpt.save_checkpoint(step, model, optimizer, {"epoch": 3}, storage_type=StorageType.MEMORY)
    >>> extra = ckpt.load_checkpoint(model, optimizer)

    The persisted ``{checkpoint_dir}/{step}`` directory is a standard DCP
    checkpoint with top-level keys ``model``, ``optim`` and the extras.
    """

    def __init__(self, checkpoint_dir: str, comm_backend="", deletion_strategy=None,
                 save_timeout=CheckpointConstant.SAVE_TIMEOUT, replica_count=0, storage=None):
        self.checkpoint_dir = checkpoint_dir
        self.storage = storage or get_checkpoint_storage(deletion_strategy)
        self._engine = FsdpCheckpointEngine(checkpoint_dir, self.storage, comm_backend, save_timeout,
                                            replica_count=replica_count)

    @property
    def engine(self):
        return self._engine

    def _state(self, model, optimizer, extra_sd):
        msd, osd = _model_optim_state(model, optimizer, full=False)
        sd = {"model": msd}
        if osd is not None:
            sd["optim"] = osd
        sd.update(extra_sd or {})
        return sd

    def prepare(self, model, optimizer, extra_sd=None) -> bool:
        """Start the one-time shm set-up (segment + prefault + pin of both
        slots) for this model / optimizer in the background, e.g. right after
        the first optimizer step (``CheckpointEngine.prepare_memory``)."""
        sd = self._state(model, optimizer, extra_sd)
        _, _, payload = self._engine._payload(sd)
        payload.pop("_views", None)
        return self._engine.prepare_memory({DCP_KEY: payload})

    def save_checkpoint(self, step, model, optimizer, extra_sd=None, path="", storage_type=StorageType.DISK):
        path = path or os.path.join(self.checkpoint_dir, str(step))
        if storage_type == StorageType.MEMORY and self._engine.precheck_skip():
            return False  # previous snapshot still flushing: do not even build the DCP payload
        sd = self._state(model, optimizer, extra_sd)
        paths = {DCP_KEY: path}
        if storage_type == StorageType.MEMORY:
            return self._engine.save_to_memory(step, sd, paths)
        if storage_type == StorageType.DISK:
            return self._engine.save_to_storage(step, sd, paths)
        raise ValueError(f"unsupported storage type {storage_type}")

    def load_checkpoint(self, model, optimizer, resume_path="", extra_sd=None):
        """Restore model/optimizer in place; returns the extras (with their
        saved values) plus ``"step"``, or ``{}`` if there is no checkpoint.

        ``extra_sd``: template of the extra entries that were saved (needed
        when restoring from storage, where DCP loads only requested keys)."""
        sd = self._state(model, optimizer, extra_sd)
        step = self._engine.load_into(sd, resume_path)
        if step == 0:
            return {}
        _set_model_optim_state(model, optimizer, sd.pop("model"), sd.pop("optim", None), full=False)
        sd["step"] = step
        return sd

    def wait_latest_checkpoint(self, timeout=1800):
        self._engine.wait_for_memory_save()

    def close(self):
        self._engine.close()


class FsdpFullCheckpointer(Checkpointer):
    """Full (unsharded) state: every rank gathers the full model/optimizer
    state and one node copy is snapshotted split across the local ranks;
    persisted as ``{dir}/{step}/rank_0.pt`` (plain ``torch.save``).
    Reference ``fsdp.py:152-290``."""

    def __init__(self, checkpoint_dir: str, comm_backend="", deletion_strategy=None,
                 save_timeout=CheckpointConstant.SAVE_TIMEOUT, storage=None):
        self.checkpoint_dir = checkpoint_dir
        self._rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.storage = storage or get_checkpoint_storage(deletion_strategy)
        self._engine = FullCheckpointEngine(checkpoint_dir=checkpoint_dir, storage=self.storage,
                                            local_shard_num=1, global_shard_num=1, comm_backend=comm_backend,
                                            save_timeout=save_timeout)

    @property
    def engine(self):
        return self._engine

    def save_checkpoint(self, step, model, optimizer, extra_sd=None, path="", storage_type=StorageType.DISK):
        path = path or os.path.join(self.checkpoint_dir, f"{step}/rank_0.pt")
        msd, osd = _model_optim_state(model, optimizer, full=True)
        sd = {"model": msd, "optimizer": osd}
        sd.update(extra_sd or {})
        sd = {CheckpointConstant.MODEL_STATES_NAME: sd}
        paths = {CheckpointConstant.MODEL_STATES_NAME: path}
        if storage_type == StorageType.MEMORY:
            return self._engine.save_to_memory(step, sd, paths)
        if storage_type == StorageType.DISK:
            return self._engine.save_to_storage(step, sd, paths)
        raise ValueError(f"unsupported storage type {storage_type}")

    def load_checkpoint(self, model, optimizer, resume_path=""):
        state = self._engine.load(resume_path)
        if not state:
            return {}
        state = dict(state)
        msd = state.pop("model", {})
        osd = state.pop("optimizer", None)
        _set_model_optim_state(model, optimizer, msd, osd, full=True)
        return state

    def wait_latest_checkpoint(self, timeout=1800):
        self._engine.wait_for_memory_save()

    def close(self):
        self._engine.close()


def wait_for_persist(checkpoint_dir: str, step: int, timeout: float = 120.0) -> bool:
    """Poll the tracker file until ``step`` is committed (tests/tools)."""
    tracker = os.path.join(checkpoint_dir, CheckpointConstant.TRACER_FILE_NAME)
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            with open(tracker) as f:
                if f.read().strip() == str(step):
                    return True
        except FileNotFoundError:
            pass
        time.sleep(0.05)
    return False
