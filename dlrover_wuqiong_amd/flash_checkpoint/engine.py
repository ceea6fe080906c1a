"""Trainer-side flash-checkpoint engine.

Runs inside every training process.  ``save_to_memory`` snapshots the state
dict into the node's shared memory (see ``copier.py`` for the GPU data path)
and returns as soon as the GPU snapshot kernel is enqueued; the agent (or a
local saver thread when not launched by ``dwamd-run``) persists shm to
storage asynchronously.  ``load`` restores from shm when every rank holds the
same complete step, otherwise from storage.

Parity: reference ``dlrover/trainer/torch/flash_checkpoint/engine.py``
(``CheckpointEngine`` :136-435, ``check_all_rank_ready`` :53,
``verify_all_rank_step_consistent`` :70, ``start_saver_process`` :114) and
``full_ckpt_engine.py`` (``FullCheckpointEngine``).

Replicated vs sharded state:
 * ``replicated=True`` (DDP): the node holds ONE copy; each of the L local
   ranks snapshots and flushes 1/L of it (parallel PCIe links), and restore
   H2D's 1/L per rank + RCCL all-gather over xGMI.
 * ``replicated=False`` (FSDP/ZeRO/Megatron shards): one segment per local
   rank, each rank moves its own shard.
"""

import gc
import hashlib
import os
import threading
import time
from abc import ABC, abstractmethod
from datetime import timedelta
from typing import Any, Dict, List, Optional

import torch
import torch.distributed as dist

from ..common import env_utils
from ..common.constants import CheckpointConstant
from ..common.log import logger
from ..common.multi_process import SharedLock, SharedQueue
from ..common.serialize import ClassMeta
from ..common.storage import CheckpointStorage, get_checkpoint_storage
from .layout import Layout, TensorMeta, iter_leaves, plan_layout, split_ranges, traverse
from .shm_handler import (DLROVER_CKPT_CONFIG_KEY, EVENT_QUEUE_SIZE, CheckpointConfig,
                          CheckpointSharedObjPrefix, SharedMemoryHandler, slot_lock_name)


_TIMING = os.environ.get("DWAMD_CKPT_TIMING", "0") == "1"  # log per-phase save times
_PREP_PIECE = max(64, int(os.environ.get("DWAMD_PREP_PIECE_MB", "1024"))) << 20  # shm prefault/pin granularity



# DWAMD_CKPT_SPECULATE=0: walk + verify the state dict before enqueueing the copy
_SPECULATE = os.environ.get("DWAMD_CKPT_SPECULATE", "1") == "1"

class CheckpointEventType:
    SAVE = 1
    UPDATE_SHARD = 2
    EXIT = 3


class CheckpointEvent:
    def __init__(self, type=CheckpointEventType.SAVE, step=0, global_shard_num=0):
        self.type = type
        self.step = step
        self.global_shard_num = global_shard_num

    def __repr__(self):
        return f"CheckpointEvent(type={self.type}, step={self.step}, shards={self.global_shard_num})"


def _ctl_reduce_min(group, value: int) -> int:
    if not dist.is_available() or not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item())


def check_all_rank_ready(group, ready: bool) -> bool:
    """True iff every rank of ``group`` is ready (CPU/gloo collective: no GPU
    stream sync is needed to take the decision)."""
    return _ctl_reduce_min(group, 1 if ready else 0) == 1


def verify_all_rank_step_consistent(group, step: int) -> bool:
    if not dist.is_available() or not dist.is_initialized():
        return True
    t = torch.tensor([step, -step], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t[0]) == step and -int(t[1]) == step


def agree_on_step(group, steps: Optional[List[int]]) -> int:
    """Latest step every rank holds complete in memory (0 if none).
    ``steps=None``: this rank holds no shard and accepts any step."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return max(steps) if steps else 0
    allv: List[Optional[List[int]]] = [None] * dist.get_world_size(group)
    dist.all_gather_object(allv, None if steps is None else sorted(steps), group=group)
    common = None
    for s in allv:
        if s is None:
            continue
        common = set(s) if common is None else common & set(s)
    return max(common) if common else 0


class _LocalSaverThread:
    """When the training process was not launched by the agent, local rank 0
    hosts the asynchronous saver in a daemon thread (reference
    ``start_saver_process`` forks a process instead; a thread avoids forking
    a GPU-initialised process)."""

    started_for = None  # shm namespace the saver listens on

    @classmethod
    def ensure(cls):
        from ..common.multi_process import shm_name

        ns = shm_name("", "")
        if cls.started_for == ns or env_utils.is_under_agent():
            return
        if env_utils.get_local_rank() != 0:
            return
        from ..elastic_agent.ckpt_saver import AsyncCheckpointSaver

        AsyncCheckpointSaver.start_async_saving_ckpt()
        cls.started_for = ns


class CheckpointEngine(ABC):
    def __init__(self, checkpoint_dir: str, storage: Optional[CheckpointStorage] = None,
                 comm_backend: str = "", save_timeout: int = CheckpointConstant.SAVE_TIMEOUT,
                 replica_count: int = 0, replicated: bool = False):
        from ..elastic_agent.standby import is_standby

        if is_standby():
            # a deep standby has no rank yet: it must block in standby_point()
            # before touching the node's checkpoint (it would otherwise write
            # the live job's shm as a world-1 trainer)
            raise RuntimeError("checkpoint engine created in a deep standby before standby_point()")
        _LocalSaverThread.ensure()
        self.checkpoint_dir = checkpoint_dir
        # this job's id in the shm header: 63-bit hash of the checkpoint dir
        self._owner_id = int.from_bytes(hashlib.blake2b(os.path.realpath(checkpoint_dir or ".").encode(),
                                                        digest_size=8).digest(), "little") >> 1 or 1
        self.storage = storage or get_checkpoint_storage()
        self._save_timeout = save_timeout
        self._replicated = replicated
        self._local_rank = env_utils.get_local_rank()
        self._local_world = env_utils.get_local_world_size()
        self._rank = 0
        self._world = 1
        self._group_rank = env_utils.get_group_rank()
        if dist.is_available() and dist.is_initialized():
            self._rank = dist.get_rank()
            self._world = dist.get_world_size()
            self._local_world = min(self._local_world, self._world) or 1
        self._cached_step = 0
        self._restart_count = env_utils.get_torch_restart_count()
        self.local_shard_num = self.get_local_shard_num()
        self.local_shard_id = 0 if self._replicated else self._local_rank % max(1, self.local_shard_num)
        self._num_slices = self._local_world if self._replicated else 1
        self._slice_idx = self._local_rank if self._replicated else 0
        self._is_shard_owner = (self._local_rank == self.local_shard_id) if not self._replicated else (
            self._local_rank == 0)

        self._shm_handler = SharedMemoryHandler(self.local_shard_id, host=False)
        self._shm_locks = [SharedLock(slot_lock_name(self.local_shard_id, s), create=True)
                           for s in range(self._shm_handler.num_slots)]
        self._next_slot: Optional[int] = None
        self._event_queue = (SharedQueue(CheckpointSharedObjPrefix.SAVE_STEP_QNAME + "0", create=True,
                                         maxsize=EVENT_QUEUE_SIZE)
                             if self._local_rank == 0 else None)
        self._ctl_group = None
        self._gather_group = None
        self._gather_on_host = False
        self._init_groups(comm_backend)
        self._copier = None
        self._layout: Optional[Layout] = None
        self._layout_key = None
        self._held_slots = set()  # slots whose lock this process holds until their flush lands
        self.skipped_saves = 0  # saves skipped while the previous snapshot was still flushing
        self._gc_frozen = False
        self._generation = 0
        self._shm_prep = None  # Future: background prefault + pin of this rank's slot slices
        self._shm_handler.before_unmap = self._quiesce_shm_users
        # learn which optimizers exist from their first step on (an
        # overlapped / ring snapshot only defers copying step-only storages)
        from .copier import _install_fence_hook

        _install_fence_hook()
        self._prep_pool = None
        self._prepped_for = None
        self._last_save_blocking = 0.0
        self.last_restore_source = None  # "hbm" | "shm" | "storage" after an in-place restore
        self.last_deferred_restore = None  # deferred_restore.DeferredRestore of the last restore
        # checkpointers whose restores feed straight into training (DDP) let
        # optimizer state land behind the first step (deferred_restore.py)
        self.defer_optimizer_restore = False
        self.last_storage_load_stats: Dict[str, float] = {}
        self.speculation_misses = 0  # speculative snapshots redone after the state dict changed
        self.last_restore_breakdown: Dict[str, float] = {}  # host seconds per restore phase
        self.host_plan: Optional[dict] = None  # node host-memory plan of the shm segment(s) (hbm_budget.host_plan)
        self._notify_agent_to_create_saver()
        self._update_saver_config()
        from .replica import CkptReplicaManager

        self._replica_manager = CkptReplicaManager.create(self, replica_count)

    # ------------------------------------------------------------ groups
    def _init_groups(self, comm_backend: str):
        if not (dist.is_available() and dist.is_initialized()):
            return
        backend = dist.get_backend()
        # control collectives on CPU (gloo) so decisions never sync the GPU
        if backend == "gloo":
            self._ctl_group = None
        else:
            self._ctl_group = dist.new_group(backend="gloo", timeout=timedelta(seconds=120))
        # intra-node group for the replicated all-gather restore.  RCCL over
        # xGMI on MI355X; a gloo world (CPU rehearsal, ranks sharing one GPU)
        # takes the SAME sliced-restore branches with the gather staged through
        # pinned host memory (gather.py).  DWAMD_GLOO_GATHER=shm: the older
        # gloo-only path where slices meet in the node's shm instead.
        if self._replicated and self._local_world > 1:
            n_nodes = self._world // self._local_world
            gb = comm_backend or backend
            host_meet = gb == "gloo" and os.environ.get("DWAMD_GLOO_GATHER", "staged") == "shm"
            if n_nodes <= 1:
                self._gather_group = None if host_meet else dist.group.WORLD
            else:
                for node in range(n_nodes):
                    ranks = list(range(node * self._local_world, (node + 1) * self._local_world))
                    g = dist.new_group(ranks=ranks, backend=gb)
                    if self._rank in ranks and not host_meet:
                        self._gather_group = g
            self._gather_on_host = self._gather_group is None

    def _ctl_barrier(self):
        if dist.is_available() and dist.is_initialized():
            dist.barrier(group=self._ctl_group)

    # -------------------------------------------------------- agent notify
    def _notify_agent_to_create_saver(self):
        if self._local_rank != 0:
            return
        queue = SharedQueue("factory", create=True, maxsize=4)
        clazz = self.get_saver_class()
        meta = ClassMeta(module_path=clazz.__module__, class_name=clazz.__name__, kwargs={
            "checkpoint_dir": self.checkpoint_dir,
            "storage_meta": self.storage.get_class_meta(),
            "local_shard_num": self.local_shard_num,
            "global_shard_num": self.get_global_shard_num(),
            "save_timeout": self._save_timeout,
        })
        try:
            queue.put(meta, timeout=5)
        except Exception:
            logger.warning("saver factory queue is full; the agent already has a saver")

    def _update_saver_config(self):
        if self._local_rank == 0 and self._event_queue is not None:
            ev = CheckpointEvent(type=CheckpointEventType.UPDATE_SHARD,
                                 global_shard_num=self.get_global_shard_num())
            try:
                self._event_queue.put(ev, timeout=5)
            except Exception:
                logger.warning("checkpoint event queue full; UPDATE_SHARD dropped")

    # ------------------------------------------------------------ helpers
    def _device_copier(self):
        if self._copier is None and torch.cuda.is_available():
            from .copier import GpuCopier

            self._copier = GpuCopier(torch.device("cuda", torch.cuda.current_device()))
        return self._copier

    def _plan(self, state_dict) -> Layout:
        if not hasattr(self, "_layout_cache"):
            from .layout import LayoutCache

            self._layout_cache = LayoutCache()
        layout, tensors = self._layout_cache.plan(state_dict)
        self._keepalive = tensors
        return layout

    def _ensure_shm(self, total: int):
        """(Re)create the segment when the payload size changes.  Only the
        create/attach (ftruncate + mmap, ~ms) happens here, inside the
        training pause; prefaulting and hipHostRegister of this rank's slices
        (~1 s per 20 GB) run on a background thread that the first flush --
        not the training thread -- waits for."""
        h = self._shm_handler
        cur = h.payload_size if h.shared_memory is not None else -1
        need_resize = cur != total
        if need_resize and self._copier is not None:
            # registrations of the old mapping must not outlive it (a new
            # mmap may land on the same addresses and look pinned)
            self._copier.wait()
            if self._shm_prep is not None:
                self._shm_prep.result()
            self._copier.pinned.release_all()
        if self._replicated:
            # every local rank plans the same layout -> same decision
            if need_resize:
                self._ctl_barrier()
                if self._local_rank == 0:
                    slots = self._plan_host_memory(total, segments=1)
                    h.close()
                    h.init_shared_memory(create=True, size=total, owner=self._owner_id, slots=slots)
                self._ctl_barrier()
                if self._local_rank != 0:
                    h.close()
                    h.init_shared_memory(create=False)
                self._generation += 1
                self._next_slot = None
        elif need_resize:
            slots = self._plan_host_memory(total, segments=max(1, self.local_shard_num))
            h.close()
            h.init_shared_memory(create=True, size=total, owner=self._owner_id, slots=slots)
            self._generation += 1
            self._next_slot = None
        if need_resize:
            self._log_hbm_plan(total)
        key = (h.shared_memory.ino if h.shared_memory is not None else -1, total)
        if self._prepped_for != key:
            # new segment, or an existing one this process attached (restart):
            # make sure every slot this rank writes is pinned before its flush
            self._prepped_for = key
            self._start_shm_prep(total, prefault=need_resize)

    def _plan_host_memory(self, payload: int, segments: int) -> Optional[int]:
        """Host-memory preflight before the node's checkpoint segment(s) are
        (re)created (hbm_budget.host_plan): the slot count that fits, or a
        clean HostMemoryError instead of a SIGBUS on first touch.
        ``DWAMD_HOST_BUDGET=off`` skips it."""
        self.host_plan = None
        if os.environ.get("DWAMD_HOST_BUDGET", "on") == "off":
            return None
        import glob

        from ..common.multi_process import shm_name
        from .hbm_budget import HostMemoryError, host_plan

        prefix = shm_name("seg", CheckpointSharedObjPrefix.SHM_NAME)
        mine = 0
        for f in glob.glob("/dev/shm/" + prefix.lstrip("/") + "*"):
            try:
                mine += os.stat(f).st_blocks * 512  # pages this job's segments hold now
            except OSError:
                pass
        p = host_plan(payload, segments, want_slots=self._shm_handler.max_slots, reclaimable=mine)
        self.host_plan = p.as_dict()
        if not p.fits:
            raise HostMemoryError(f"flash checkpoint: {p.notes.get('slots')}; set DWAMD_HOST_RESERVE_GB lower, "
                                  f"free host memory or save to storage only")
        if p.notes:
            logger.warning(f"rank {self._rank}: host memory plan: {p.notes['slots']}")
        logger.info(f"rank {self._rank}: host memory plan {self.host_plan}")
        return p.slots

    def _log_hbm_plan(self, payload: int):
        """HBM-budget preflight (hbm_budget.py) for this GPU, logged once per
        payload size: staging, standby, restore-gather temporary."""
        self.hbm_plan = None
        if not torch.cuda.is_available() or payload <= 0:
            return
        try:
            from .hbm_budget import plan

            from . import copier as _cp

            dev = torch.cuda.current_device()
            _free, total = torch.cuda.mem_get_info(dev)
            state = int(torch.cuda.memory_allocated(dev))
            # gradients a deferred optimizer-state write-back would keep (ring)
            grad_bytes = sum(o.flat.grad.numel() * o.flat.grad.element_size() for o in list(_cp._OPTIMIZERS or ())
                             if getattr(o, "_dsw_supported", lambda: False)() and getattr(o, "flat", None) is not None
                             and o.flat.grad is not None)
            p = plan(total, worker_state=state, worker_peak=max(state, int(torch.cuda.max_memory_reserved(dev))),
                     payload=payload, world_local=self._num_slices if self._replicated else self._local_world,
                     replicated=self._replicated, standby=os.environ.get("DWAMD_STANDBY_MODE", "import"),
                     hbm_tier=os.environ.get("DWAMD_HBM_TIER", "1") == "1", grad_bytes=grad_bytes,
                     staging_mode=os.environ.get("DWAMD_STAGING", "auto"),
                     ring_bytes=int(float(os.environ.get("DWAMD_RING_HBM_GB", "0")) * (1 << 30)))
            self.hbm_plan = p.as_dict()
            logger.info(f"rank {self._rank}: HBM budget {self.hbm_plan}")
        except Exception as e:  # a log line must never fail a save
            logger.warning(f"HBM budget preflight skipped: {e}")

    def _quiesce_shm_users(self):
        """Before this process unmaps its segment (resize, a stale mapping
        replaced by a writer, close): the prep thread and in-flight flushes
        write into it, and pinned registrations must not outlive it."""
        if self._shm_prep is not None:
            self._shm_prep.result()
            self._shm_prep = None
            self._prepped_for = None
        if self._copier is not None:
            self._copier.wait()
            # a deferred optimizer-state restore still DMAs from this
            # segment's pinned pages on its side stream: let it land first
            from . import deferred_restore

            deferred_restore.synchronize_all()
            self._copier.pinned.release_all()

    def _start_shm_prep(self, total: int, prefault: bool):
        copier = self._device_copier()
        h = self._shm_handler
        if total <= 0 or h.shared_memory is None:
            return
        lo, hi = split_ranges(total, self._num_slices)[self._slice_idx]
        # the slot the next save writes first: its flush waits only for that
        # slot's prefault + registration, not for the whole segment's
        first = self._next_slot if self._next_slot is not None else h.write_slot()
        order = [first] + [s for s in range(h.num_slots) if s != first]
        ranges = [(h.payload_addr(slot) + lo, hi - lo) for slot in order]
        from .copier import PrepTracker

        tracker = PrepTracker()
        futs = [tracker.add(a, n) for a, n in ranges]
        first_done = futs[0]
        piece = _PREP_PIECE

        def prep():
            import ctypes

            from .._native import runtime

            t0 = time.perf_counter()
            try:
                for i, (addr, n) in enumerate(ranges):
                    # piecewise: populating / registering tens of GB in one
                    # call holds this process's mm lock for seconds, and every
                    # HIP allocation of the training thread queues behind it
                    for o in range(0, n, piece):
                        c = min(piece, n - o)
                        if prefault:
                            runtime().dw_prefault(ctypes.c_void_p(addr + o), c, 1)
                        if copier is not None:
                            copier.pinned.ensure(addr + o, c)
                        time.sleep(0.001)  # let a waiting mm writer in
                    futs[i].set_result(time.perf_counter() - t0)
            finally:
                tracker.fail_pending()
            if _TIMING:
                logger.info(f"shm prep ({len(ranges)} slot slices, {hi - lo} B each): first slot "
                            f"{1000 * (first_done.result() or 0):.1f} ms, all {1000 * (time.perf_counter() - t0):.1f} ms "
                            "(background)")

        from concurrent.futures import ThreadPoolExecutor

        if self._prep_pool is None:
            self._prep_pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="dwamd-shm-prep")
        self._shm_prep = self._prep_pool.submit(prep)
        if copier is not None:
            copier.pending_prep = tracker

    # ----------------------------------------------------------- core save
    def save_state_dict_to_memory(self, state_dict: Dict, conf: CheckpointConfig) -> bool:
        # The training pause must not absorb a full (generation-2) Python GC
        # pass, which with a model's worth of tensors, layouts and meta trees
        # costs ~90 ms: collection is deferred past the snapshot, and after the
        # first save every long-lived object (model, optimizer, cached layout)
        # is frozen out of future full collections.
        enabled = gc.isenabled()
        gc.disable()
        try:
            return self._save_state_dict_to_memory(state_dict, conf)
        finally:
            if not self._gc_frozen:
                gc.freeze()
                self._gc_frozen = True
            if enabled:
                gc.enable()
            # under the agent: record what a replacement's first step needs
            # (GEMMs of the next optimizer step + allocator peak) for the
            # import-mode standby to replay (elastic_agent/warm_profile.py)
            from ..elastic_agent import warm_profile

            # (the snapshot staging this process allocated is not part of
            # the footprint a standby reserves: it holds its own staging)
            c = self._copier
            warm_profile.on_save(sum(t.numel() for t in c._stagings if isinstance(t, torch.Tensor))
                                 if c is not None else 0)

    def _skip_busy(self) -> bool:
        """Reference semantics (a save is skipped while the previous one is
        still being written): skip when the staging buffer this snapshot needs
        is still flushing and would not be free within DWAMD_CKPT_MAX_WAIT_MS
        (``DWAMD_CKPT_BUSY=wait`` blocks instead).  Decided collectively so
        every rank skips the same saves."""
        if os.environ.get("DWAMD_CKPT_BUSY", "skip") != "skip" or getattr(self, "_storage_save", False):
            return False
        c = self._copier
        eta = c.stage_busy_eta() if c is not None else 0.0
        busy = 1 if eta * 1000.0 > float(os.environ.get("DWAMD_CKPT_MAX_WAIT_MS", "250")) else 0
        if dist.is_available() and dist.is_initialized() and self._ctl_group is not None:
            t = torch.tensor([busy], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._ctl_group)
            busy = int(t)
        if busy:
            self.skipped_saves += 1
            if self.skipped_saves <= 3 or self.skipped_saves % 50 == 0:
                logger.info(f"rank {self._rank}: memory checkpoint skipped, the previous one is still being "
                            f"written to shm ({self.skipped_saves} skipped so far)")
        return bool(busy)

    def precheck_skip(self) -> bool:
        """Collective busy check a checkpointer runs BEFORE building an
        expensive state dict (FSDP DCP payload); the save that follows does
        not vote again."""
        skip = self._skip_busy()
        self._prechecked = not skip
        return skip

    def prepare_memory(self, state_dict: Dict) -> bool:
        """Start the one-time shm set-up for ``state_dict`` now, in the
        background: create the segment and prefault + hipHostRegister this
        rank's slot slices (~15 GB/s of host page zeroing: a 124 GB TP-shard
        checkpoint needs ~16 s for its two slots).  Call it once the model and
        the optimizer state exist -- it then overlaps the first training steps
        instead of delaying the first save's flush.  Collective for replicated
        engines (same call on every local rank).  Returns False for ranks that
        never save (data-parallel replicas of a shard)."""
        if not self._replicated and self._local_rank != self.local_shard_id:
            return False
        layout = self._plan(state_dict)
        if layout.total_bytes <= 0:
            return False
        self._ensure_shm(layout.total_bytes)
        return True

    def _save_state_dict_to_memory(self, state_dict: Dict, conf: CheckpointConfig) -> bool:
        if getattr(self, "_prechecked", False):
            self._prechecked = False
        elif self._skip_busy():
            return False
        if not self._replicated and self._local_rank != self.local_shard_id:
            # not a saving rank (e.g. a data-parallel replica of a TP/PP shard):
            # still takes part in the slot vote of the saving ranks
            if dist.is_available() and dist.is_initialized():
                t = torch.ones(self._shm_handler.max_slots, dtype=torch.int64)
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self._ctl_group)
            return False
        t0 = time.perf_counter()
        marks = [("start", t0)] if _TIMING else None
        copier = self._device_copier()
        if copier is not None:
            # only the flush that used the staging buffer (and shm slot) this
            # snapshot reuses; with double staging the previous one may still run
            copier.wait_stage()
        if self._next_slot is not None:
            self._wait_own_lock_release(slot=self._next_slot)
        if marks is not None:
            marks.append(("wait_prev", time.perf_counter()))

        h = self._shm_handler
        step = conf.step
        stage = {}

        def before_copy(idx: int):
            # HBM tier: this staging buffer is about to be overwritten
            stage["idx"] = idx
            h.set_hbm_stamp(self._slice_idx, idx, 0)

        def can_snapshot(lay) -> bool:
            lo_, hi_ = split_ranges(lay.total_bytes, self._num_slices)[self._slice_idx]
            return (copier is not None and bool(state_dict) and any(e.device == "cuda" for e in lay.extents)
                    and not copier._use_ring(hi_ - lo_))

        snap = None
        # Speculative snapshot: a training loop saves the same tensors every
        # time, so the HBM->staging copy is enqueued from the previous plan
        # (whose tensors this engine still holds: every address stays valid)
        # BEFORE the state dict is walked and verified against it (~3-5 ms of
        # host time for a few thousand tensors, now overlapped with the copy).
        # A mismatch re-plans and copies again (stream-ordered after it).
        spec = self._layout_cache.cached() if (hasattr(self, "_layout_cache") and _SPECULATE) else None
        if spec is not None and h.shared_memory is not None and h.payload_size == spec.total_bytes \
                and can_snapshot(spec):
            lo, hi = split_ranges(spec.total_bytes, self._num_slices)[self._slice_idx]
            snap = copier.snapshot(spec, lo, hi, before_copy)
            if marks is not None:
                marks.append(("enqueue", time.perf_counter()))
        layout = self._plan(state_dict)
        if snap is not None and layout.extents is not spec.extents:
            self.speculation_misses += 1
            if "idx" in stage:
                # redo into the SAME staging buffer: the other one still holds
                # the previous complete step (HBM-tier recovery stays possible)
                copier.rewind_stage(stage["idx"])
            stage.clear()
            snap = None  # the speculative copy is stream-ordered before the real one below
        self._ensure_shm(layout.total_bytes)
        if marks is not None:
            marks.append(("plan+shm", time.perf_counter()))
        lo, hi = split_ranges(layout.total_bytes, self._num_slices)[self._slice_idx]
        has_gpu = any(e.device == "cuda" for e in layout.extents)
        if snap is None and can_snapshot(layout):
            # the HBM->staging copy needs no shm slot: enqueue it first, so the
            # slot vote (a gloo collective) and the metadata pickling below run
            # on the host while the GPU copies
            snap = copier.snapshot(layout, lo, hi, before_copy)
            if marks is not None:
                marks.append(("enqueue", time.perf_counter()))
        elif snap is not None:
            snap["layout"] = layout  # same extents; the verified meta tree
        if self._next_slot is None:
            # first save of this process (nothing in flight): never the latest complete slot
            self._next_slot = h.write_slot()
        slot = self._choose_slot(h, bool(state_dict))
        if marks is not None:
            marks.append(("slot", time.perf_counter()))
        if slot < 0:
            logger.info(f"rank {self._rank} skips the memory checkpoint of step {conf.step}: "
                        "its shm slots are busy (the agent persisting them, a replica transfer, or the "
                        "previous flush)")
            return False
        if self._is_shard_owner:
            self._held_slots.add(slot)
        self._next_slot = (slot + 1) % h.num_slots

        conf.rank = self._rank
        conf.group_rank = self._group_rank
        conf.world_size = self._world
        conf.num_slices = self._num_slices
        conf.generation = self._generation
        h.set_slice_step(slot, self._slice_idx, 0)  # slot reads incomplete before any byte changes
        if self._is_shard_owner:
            h.set_metadata(slot, layout.meta_tree, conf)

        def on_snapshot():
            if "idx" in stage:
                # the (standby-owned) staging buffer holds the whole slice of
                # ``step``: recoverable even if this process dies mid-flush
                h.set_hbm_stamp(self._slice_idx, stage["idx"], step, copier.stage_owner(stage["idx"]), hi - lo)

        def on_done():
            h.set_slice_step(slot, self._slice_idx, step)
            if "idx" in stage:
                # the staging buffer now holds exactly the bytes of the slice
                # that just became complete in shm
                h.set_hbm_stamp(self._slice_idx, stage["idx"], step, copier.stage_owner(stage["idx"]), hi - lo)
            if self._is_shard_owner:
                self._release_when_complete(step, slot)

        if snap is not None:
            copier.flush_snapshot(snap, h.payload_addr(slot), on_done, on_snapshot=on_snapshot)
        elif has_gpu and copier is not None:
            copier.save_slice(layout, h.payload_addr(slot), lo, hi, on_done, before_copy=before_copy,
                              on_snapshot=on_snapshot)
        else:
            self._cpu_save_slice(layout, h.payload_addr(slot), lo, hi)
            on_done()
        self._cached_step = step
        self._last_save_blocking = time.perf_counter() - t0
        if marks is not None:
            marks.append(("snapshot", time.perf_counter()))
            logger.info("ckpt save phases (ms): " + ", ".join(
                f"{n}={1000 * (t - marks[i][1]):.1f}" for i, (n, t) in enumerate(marks[1:])))
        self._replica_manager.backup(self._shm_handler)
        return True

    def _choose_slot(self, h: SharedMemoryHandler, has_state: bool) -> int:
        """Slot this save writes (same on every rank), its lock held by the
        shard owner; -1 = skip.  Preferred: the alternating ``_next_slot``.
        If the agent holds it (persisting), the other slot is used provided
        an intact complete checkpoint remains (the one being persisted).
        Shard owners vote with per-slot flags (gloo MIN) so all ranks agree."""
        n = h.num_slots
        order = [self._next_slot] + [s for s in range(n) if s != self._next_slot]
        # the vote always carries max_slots flags (a 1-slot segment marks the
        # rest unusable): every rank's tensor has the same shape
        flags = [1] * n + [0] * (h.max_slots - n)
        acquired = {}
        if self._is_shard_owner:
            complete = h.complete_steps()
            complete_slots = set(complete.values())
            for s in order:
                others_intact = any(c in complete_slots for c in range(n) if c != s)
                allowed = s == self._next_slot or others_intact or not complete_slots
                ok = allowed and has_state and self._shm_locks[s].acquire(blocking=False)
                flags[s] = 1 if ok else 0
                if ok:
                    acquired[s] = True
        elif not has_state:
            flags = [0] * h.max_slots
        if dist.is_available() and dist.is_initialized():
            t = torch.tensor(flags, dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self._ctl_group)
            flags = [int(x) for x in t]
        slot = next((s for s in order if flags[s]), -1)
        for s in acquired:
            if s != slot:
                self._shm_locks[s].release()
        return slot

    def _cpu_save_slice(self, layout: Layout, base: int, lo: int, hi: int):
        import ctypes

        from .._native import runtime
        from .layout import intersect_extents

        for e, a, b in intersect_extents(layout.extents, lo, hi):
            if e.device == "cuda":
                # no copier (should not happen on a GPU host): go through torch
                t = e.keepalive
                raise RuntimeError("GPU tensors in state dict but no GPU copier available")
            runtime().dw_memcpy_parallel(ctypes.c_void_p(base + a), ctypes.c_void_p(e.src_ptr + (a - e.offset)),
                                         b - a, 8)

    def _release_when_complete(self, step: int, slot: int):
        """Shard owner: keep the slot lock until every slice holds ``step``."""
        if slot not in self._held_slots:
            return
        h = self._shm_handler
        deadline = time.time() + self._save_timeout

        def _wait():
            while time.time() < deadline:
                if all(s == step for s in h.slice_steps(slot, self._num_slices)):
                    break
                time.sleep(0.0005)
            self._held_slots.discard(slot)
            self._shm_locks[slot].release()

        if self._num_slices <= 1:
            _wait()
        else:
            threading.Thread(target=_wait, daemon=True, name="dwamd-ckpt-unlock").start()

    def _wait_own_lock_release(self, timeout: float = 600.0, slot: Optional[int] = None):
        """Wait until this process no longer holds ``slot``'s lock (any slot
        when None), i.e. the snapshot written there has fully landed."""
        deadline = time.time() + timeout
        while time.time() < deadline and (self._held_slots if slot is None else slot in self._held_slots):
            time.sleep(0.0005)

    def snapshot_fence(self):
        """Order the current stream after a pending overlapped snapshot
        (``DWAMD_OVERLAP_SNAPSHOT=1``).  Optimizer steps do this themselves
        (global step pre-hook); call it before writing checkpointed tensors
        any other way between a save and the next optimizer step."""
        c = getattr(self, "_copier", None)
        if c is not None:
            c.fence()

    def wait_for_memory_save(self):
        """Block until this process's last snapshot is in shm."""
        if self._copier is not None:
            self._copier.wait()
        self._wait_own_lock_release()

    # ----------------------------------------------------------- core load
    def _hbm_only_steps(self) -> Dict[int, int]:
        """{step: shm slot holding its metadata} of snapshots whose slice of
        this rank sits complete in an HBM-tier buffer this process owns while
        their shm flush never finished (the previous worker died mid-flush).
        GPU bytes come from HBM; metadata and CPU tensors were written to the
        slot synchronously at save time."""
        from . import hbm_tier

        if not hbm_tier.OWNED or os.environ.get("DWAMD_HBM_TIER", "1") != "1":
            return {}
        if self._replicated and self._num_slices > 1 and self._gather_group is None and not self._gather_on_host:
            return {}  # no way to combine the slices: every byte from shm
        h = self._shm_handler
        t0 = time.perf_counter()
        sub = self.hbm_scan_breakdown = {}
        if h.shared_memory is None and not h.init_shared_memory(create=False):
            return {}
        sub["attach"] = round(time.perf_counter() - t0, 4)
        complete = h.complete_steps()
        out = {}
        metas = {}
        for b in range(min(2, len(hbm_tier.OWNED))):
            st, pid, _nb = h.hbm_stamp(self._slice_idx, b)
            if st <= 0 or pid != os.getpid() or st in complete:
                continue
            from .shm_handler import META_WORDS

            hdr = getattr(h, "_header", None)
            for s in range(h.num_slots):
                # the slot's header step word (written with its metadata at
                # save time) names the candidate: unpickle only that slot's
                # metadata, not every slot's
                if hdr is not None and int(hdr[META_WORDS + 2 * s]) not in (0, st):
                    continue
                if s not in metas:
                    t1 = time.perf_counter()
                    metas[s] = h.get_meta(s)
                    sub[f"meta{s}"] = round(time.perf_counter() - t1, 4)
                cfg = metas[s].get(DLROVER_CKPT_CONFIG_KEY)
                if cfg is not None and cfg.step == st and cfg.num_slices == self._num_slices:
                    out[st] = s
        self._scanned_metas = metas  # reused by the restore that follows
        return out

    def get_state_dict_from_memory(self, target: Any = None):
        """Returns (step, state_dict) from shm, or (0, {}).

        A restart's restore is the first allocation-heavy Python work of a
        fresh process (unpickled meta trees, leaf lists) next to a model's
        worth of live objects: a 0.12-0.21 s stall moved between its
        Python-only phases from run to run (``hbm_scan.meta1``,
        ``copy_enqueue.match``), the signature of a generation-2 collection.
        Collection is deferred past the restore, and everything alive then
        (model, optimizer, restored state) is frozen out of later full
        collections, as after a save.  ``DWAMD_RESTORE_GC=1`` keeps the
        collector on (A/B)."""
        if os.environ.get("DWAMD_RESTORE_GC", "0") == "1":
            return self._get_state_dict_from_memory(target)
        enabled = gc.isenabled()
        gc.disable()
        try:
            return self._get_state_dict_from_memory(target)
        finally:
            if not self._gc_frozen:
                gc.freeze()
                self._gc_frozen = True
            if enabled:
                gc.enable()
            from .deferred_init import release_gc

            release_gc()  # a restart's model build held the collector off (deferred_init.hold_gc)

    def _get_state_dict_from_memory(self, target: Any = None):
        t0, c0 = time.perf_counter(), time.thread_time()
        self._restore_t0 = t0
        tb = self.last_restore_breakdown = {}
        # other threads alive in this process during the restore (a phase
        # whose wall time far exceeds its own CPU time was blocked: lock,
        # GIL or the mm lock a concurrent hipHostRegister holds)
        tb["threads"] = sorted(t.name for t in threading.enumerate() if t is not threading.current_thread())

        def lap(name):
            nonlocal t0, c0
            t1, c1 = time.perf_counter(), time.thread_time()
            tb[name] = round(t1 - t0, 4)
            if t1 - t0 > 0.01:
                tb["cpu." + name] = round(c1 - c0, 4)
            t0, c0 = t1, c1

        self._restore_memory_from_replica()
        h = self._shm_handler
        holds = self._replicated or self._local_rank == self.local_shard_id
        complete = h.complete_steps() if holds else {}
        foreign = bool(complete) and h.owner() not in (0, self._owner_id)
        if foreign:
            # another job's checkpoint in this shm namespace (same shard
            # name, different checkpoint dir): not ours to restore; detach so
            # the first save re-creates the segment under this job
            logger.warning(f"rank {self._rank}: shm {h.shm_name} holds another job's checkpoints "
                           f"(steps {sorted(complete)}); ignored")
            self._quiesce_shm_users()
            h.close()
            complete = {}
        lap("scan_slots")
        # a snapshot still in (standby-owned) HBM when the last worker died
        # counts too -- only for an in-place GPU restore
        hbm_only = self._hbm_only_steps() if (holds and target is not None and not foreign) else {}
        out = self._restore_step(h, holds, complete, hbm_only, target, lap, tb)
        if out is None:
            # the agreed step existed only in HBM and some rank's targets
            # cannot take the D2D path: the newest step complete in shm
            out = self._restore_step(h, holds, complete, {}, target, lap, tb)
        return out if out is not None else (0, {})

    def _restore_step(self, h, holds, complete, hbm_only, target, lap, tb):
        """Agree on a step among the candidates and restore it.  None: the
        step was HBM-only and the in-place restore was refused (collective)."""
        cands = dict(hbm_only)
        cands.update(complete)
        lap("hbm_scan")
        for k, v in (getattr(self, "hbm_scan_breakdown", None) or {}).items():
            tb["hbm_scan." + k] = v
        step = agree_on_step(self._ctl_group, list(cands) if holds else None)
        slot = cands.get(step, -1) if (step > 0 and holds) else -1
        if step <= 0 or not check_all_rank_ready(self._ctl_group, slot >= 0 or not holds):
            return 0, {}
        lap("agree")
        if not holds:
            # mirror the holders' collective votes in _restore_into
            if target is not None and self._vote_retry(not check_all_rank_ready(self._ctl_group, True), False):
                return None
            return 0, {}
        from_hbm_only = step not in complete
        logger.info(f"rank {self._rank}: restoring step {step} from memory slot {slot} "
                    f"(complete in memory: {sorted(complete)}"
                    f"{', in HBM only: ' + str(sorted(hbm_only)) if hbm_only else ''})")
        scanned = getattr(self, "_scanned_metas", None) or {}
        self._scanned_metas = None
        tree = (scanned.get(slot) or h.get_meta(slot))["tree"]
        lap("meta")
        if target is not None:
            sd = self._restore_into(tree, target, slot, step, require_hbm=from_hbm_only, lap=lap)
            lap("copy_enqueue")
            if self._vote_retry(sd is None, from_hbm_only):
                return None
            if sd is not None:
                return step, sd
        if from_hbm_only:
            return 0, {}  # never serve an incomplete shm slot
        sd = h.load_state_dict(slot)
        if isinstance(sd, dict):
            sd.pop(DLROVER_CKPT_CONFIG_KEY, None)
        return step, sd

    def _vote_retry(self, refused: bool, hbm_only: bool) -> bool:
        """After a (collectively) refused in-place restore: retry with the
        shm-complete steps only if the refused step was HBM-only on any rank.
        ``refused`` is the same on every rank, so the vote is skipped by all
        or taken by all."""
        if not refused:
            return False
        v = 1 if hbm_only else 0
        if dist.is_available() and dist.is_initialized():
            t = torch.tensor([v], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._ctl_group)
            v = int(t)
        return v == 1

    def _hbm_source(self, step: int, lo: int, hi: int) -> Optional[int]:
        """Device address of an HBM-tier buffer owned by this process that
        holds payload bytes [lo, hi) of ``step`` (see hbm_tier.py)."""
        from . import hbm_tier

        if not hbm_tier.OWNED or os.environ.get("DWAMD_HBM_TIER", "1") != "1":
            return None
        h = self._shm_handler
        for b, buf in enumerate(hbm_tier.OWNED[:2]):
            st, pid, nb = h.hbm_stamp(self._slice_idx, b)
            if st == step and pid == os.getpid() and nb == hi - lo and buf.ptr and buf.nbytes >= nb:
                return buf.ptr
        return None

    def _restore_into(self, tree, target, slot: int, step: int = 0, require_hbm: bool = False, lap=None):
        """Fast path: H2D (sliced + all-gather for replicated) straight into
        the live tensors of ``target`` (same structure as the saved dict).
        ``require_hbm``: the shm slot is incomplete -- every rank must copy
        its slice from its HBM-tier buffer.  ``lap``: phase timer of the
        caller (sub-phases ``copy_enqueue.*``)."""
        from .copier import match_targets

        lap = lap or (lambda name: None)
        pairs, ok = match_targets(tree, target)
        lap("copy_enqueue.match")
        if require_hbm:
            # the shm slot never received this step's GPU bytes: every tensor
            # saved from the GPU must land in a contiguous GPU target (the
            # D2D path from the HBM buffer); otherwise refuse on every rank
            total = self._shm_handler.payload_size
            s_lo, s_hi = split_ranges(total, self._num_slices)[self._slice_idx]
            ok = ok and self._hbm_source(step, s_lo, s_hi) is not None and all(
                t.is_cuda and t.is_contiguous() for m, t in pairs if m.device == "cuda" and m.numel > 0)
        ok_all = check_all_rank_ready(self._ctl_group, ok)
        lap("copy_enqueue.vote")
        if not ok_all:
            return None
        h = self._shm_handler
        base = h.payload_addr(slot)
        gpu_pieces, late_pieces = [], []
        late = self._late_leaf_flags(tree)
        for i, (m, t) in enumerate(pairs):
            if m.numel == 0:
                continue
            # tensors saved from the CPU were written to shm synchronously at
            # save time and are never in the HBM staging buffers: shm always
            if t.is_cuda and t.is_contiguous() and m.device == "cuda":
                (late_pieces if late and late[i] else gpu_pieces).append(
                    (m.offset, t.data_ptr(), m.numel * m.element_size))
            else:
                src = torch.frombuffer(h.shared_memory.buf, dtype=m.dtype, count=m.numel,
                                       offset=m.offset + h.payload_offset(slot))
                with torch.no_grad():
                    t.copy_(src.view(t.shape))
        total = h.payload_size
        lap("copy_enqueue.pieces")
        copier = self._device_copier() if (gpu_pieces or late_pieces) else None
        lap("copy_enqueue.copier")
        if copier is None:
            self.last_restore_source = "shm"  # host tensors: copied straight from the slot
            it = iter([t for _, t in pairs])
            return traverse(tree, lambda v: next(it) if isinstance(v, TensorMeta) else v)
        s_lo, s_hi = split_ranges(total, self._num_slices)[self._slice_idx]
        hbm_src = self._hbm_source(step, s_lo, s_hi) if step > 0 else None
        lap("copy_enqueue.hbm_source")
        self.last_restore_source = "hbm" if hbm_src is not None else "shm"
        self.last_deferred_restore = None
        if late_pieces and (hbm_src is not None or self._num_slices > 1):
            # D2D restores take milliseconds and sliced ones meet in one
            # gather: only a single-slice restore from host shm defers
            gpu_pieces, late_pieces = gpu_pieces + late_pieces, []
        if self._replicated and self._num_slices > 1 and self._gather_group is not None:
            per = split_ranges(total, self._num_slices)[0][1]
            lo = self._slice_idx * per
            copier.restore(gpu_pieces, base, total, lo, lo + per, self._gather_group, self._num_slices,
                           hbm_src=hbm_src)
        elif self._num_slices <= 1:
            copier.restore(gpu_pieces, base, total, 0, total, hbm_src=hbm_src)
            if late_pieces:
                self.last_deferred_restore = copier.restore_deferred(late_pieces, base, self._restore_t0)
        else:
            # replicated, no device all-gather (gloo world): slices meet in
            # shm.  An HBM-only step is first written back slice by slice
            # from each rank's HBM buffer (completing the shm slot), then
            # every rank reads the whole payload from shm.
            if require_hbm:
                if hbm_src is not None:
                    # the device region of this slice only: host tensors were
                    # written to shm at save time and lie after it
                    dev_end = max((m.offset + m.nbytes for m, _t in pairs if m.device == "cuda"), default=0)
                    copier.write_back(hbm_src, base + s_lo, max(0, min(s_hi, dev_end) - s_lo))
                    h.set_slice_step(slot, self._slice_idx, step)
                self._ctl_barrier()
                self.last_restore_source = "hbm->shm"
            else:
                self.last_restore_source = "shm"
            copier.restore(gpu_pieces, base, total, 0, total)
        it = iter([t for _, t in pairs])

        def pick(v):
            if isinstance(v, TensorMeta):
                return next(it)
            return v

        return traverse(tree, pick)

    def _late_leaf_flags(self, tree):
        """Per TensorMeta leaf of ``tree`` (``iter_leaves`` order, as in
        ``match_targets``): may it land after the restore returns
        (``deferred_restore``: optimizer state -- a dict key naming it in the
        first two levels, e.g. ``{"model_states": {"optimizer": ...}}``)?
        None: nothing deferrable, or the checkpointer did not opt in."""
        from . import deferred_restore

        if not (self.defer_optimizer_restore and isinstance(tree, dict) and deferred_restore.enabled()
                and torch.cuda.is_available()):
            return None
        flags = []

        def walk(v, late, depth):
            if isinstance(v, dict):
                for k, x in v.items():
                    walk(x, late or (depth < 2 and deferred_restore.is_deferred_key(k)), depth + 1)
            elif isinstance(v, (list, tuple)) and not hasattr(v, "_fields"):
                for x in v:
                    walk(x, late, depth + 1)
            elif isinstance(v, TensorMeta):
                flags.append(late)

        walk(tree, False, 0)
        return flags if any(flags) else None

    def _restore_memory_from_replica(self):
        if self._replica_manager.has_replica():
            self._replica_manager.gather(self._shm_handler)

    # --------------------------------------------------------- properties
    @property
    def last_save_blocking_sec(self) -> float:
        return self._last_save_blocking

    def close(self):
        try:
            self._replica_manager.close()
            if self._shm_prep is not None:
                self._shm_prep.result()
            if self._prep_pool is not None:
                self._prep_pool.shutdown(wait=True)
                self._prep_pool = None
            if self._copier is not None:
                self._copier.wait()
                self._wait_own_lock_release(timeout=30)
                from . import deferred_restore

                deferred_restore.synchronize_all()  # late restore copies read the pinned shm
                self._copier.close()
        finally:
            self._copier = None
            self._shm_handler.close()

    # ------------------------------------------------------- abstract API
    @abstractmethod
    def get_saving_ranks(self) -> Optional[List[int]]:
        ...

    @abstractmethod
    def get_saver_class(self):
        ...

    @abstractmethod
    def get_local_shard_num(self) -> int:
        ...

    @abstractmethod
    def get_global_shard_num(self) -> int:
        ...

    @abstractmethod
    def save_to_memory(self, step, state_dict, paths: Dict[str, str]) -> bool:
        ...

    @abstractmethod
    def save_to_storage(self, step, state_dict, paths: Dict[str, str]) -> bool:
        ...

    @abstractmethod
    def load(self, resume_path: str = "", target: Any = None):
        ...

    def _notify_persist(self, step: int):
        # every node's agent persists its own local shards (node 0 also commits)
        if self._local_rank == 0 and self._event_queue is not None:
            self._event_queue.put(CheckpointEvent(type=CheckpointEventType.SAVE, step=step), timeout=60)


class FullCheckpointEngine(CheckpointEngine):
    """Replicated (DDP) state.  ``local_shard_num == 1``: one node copy split
    across local ranks; ``local_shard_num == local_world``: per-rank copies
    (reference semantics for partitioned models)."""

    def __init__(self, checkpoint_dir, storage=None, local_shard_num=1, global_shard_num=1,
                 comm_backend="", save_timeout=CheckpointConstant.SAVE_TIMEOUT, replica_count=0,
                 replicated: Optional[bool] = None):
        """``replicated=False`` with ``local_shard_num=1``: only local rank 0
        holds the state (e.g. DeepSpeed ZeRO-0 saves on rank 0 only)."""
        self._local_shard_num = max(1, local_shard_num)
        self._global_shard_num = max(global_shard_num, self._local_shard_num)
        super().__init__(checkpoint_dir, storage, comm_backend, save_timeout, replica_count,
                         replicated=(self._local_shard_num == 1) if replicated is None else replicated)

    def get_saving_ranks(self):
        return None  # every rank participates (slices)

    def get_local_shard_num(self):
        return self._local_shard_num

    def get_global_shard_num(self):
        return self._global_shard_num

    def get_saver_class(self):
        from ..elastic_agent.ckpt_saver import DdpCheckpointSaver

        return DdpCheckpointSaver

    def save_to_memory(self, step, state_dict, paths):
        conf = CheckpointConfig(step=step, paths=dict(paths))
        return self.save_state_dict_to_memory(state_dict, conf)

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

    def load(self, resume_path="", target=None):
        step, sd = self.get_state_dict_from_memory(target=target)
        if sd:
            keys = list(sd.keys())
            if len(keys) == 1:
                return sd[keys[0]]
            return sd
        return self._load_from_storage(resume_path, target)

    def _load_from_storage(self, resume_path="", target=None):
        """Persisted checkpoint -> state dict.  With ``target`` (live tensors)
        the archive streams into them (O_DIRECT parallel reads + pipelined
        H2D, ``storage_loader.py``) instead of ``torch.load`` + copy."""
        inner = target.get(CheckpointConstant.MODEL_STATES_NAME, target) if isinstance(target, dict) else None

        def read(p):
            if inner is not None and os.environ.get("DWAMD_FAST_STORAGE_LOAD", "1") == "1":
                from .storage_loader import load_archive_into

                st = {}
                try:
                    # replicated state, one file per node: each local rank
                    # reads 1/L of it and the slices meet over xGMI
                    sliced = self._replicated and self._num_slices > 1 and self._gather_group is not None
                    out = load_archive_into(p, inner, direct=os.environ.get("DWAMD_STORAGE_DIRECT", "1") == "1",
                                            stats=st, slice_idx=self._slice_idx if sliced else 0,
                                            num_slices=self._num_slices if sliced else 1,
                                            gather_group=self._gather_group if sliced else None)
                    self.last_restore_source = "storage"
                    self.last_storage_load_stats = st
                    return out
                except (KeyError, ValueError) as e:  # structure differs from the target: plain load
                    logger.info(f"fast storage load not applicable ({e}); using torch.load")
                except OSError as e:
                    if sliced:  # the peers are already in the slice all-gather: no private fallback
                        raise
                    logger.warning(f"fast storage load failed ({e}); using torch.load")
            self.last_restore_source = "storage(torch.load)"
            return torch.load(p, map_location="cpu", weights_only=True)

        if resume_path:
            return self.storage.read_state_dict(resume_path, read)
        tracker = os.path.join(self.checkpoint_dir, CheckpointConstant.TRACER_FILE_NAME)
        content = self.storage.read(tracker)
        if not content:
            return {}
        it = int(str(content).strip())
        name = "rank_0.pt" if self._global_shard_num == 1 else f"rank_{self._rank}.pt"
        return self.storage.read_state_dict(os.path.join(self.checkpoint_dir, str(it), name), read)


class ShardCheckpointEngine(FullCheckpointEngine):
    """Every rank owns a distinct shard (FSDP / ZeRO / TP-PP)."""

    def __init__(self, checkpoint_dir, storage=None, comm_backend="",
                 save_timeout=CheckpointConstant.SAVE_TIMEOUT, replica_count=0):
        lw = env_utils.get_local_world_size()
        ws = dist.get_world_size() if dist.is_available() and dist.is_initialized() else lw
        super().__init__(checkpoint_dir, storage, local_shard_num=max(lw, 1), global_shard_num=max(ws, 1),
                         comm_backend=comm_backend, save_timeout=save_timeout, replica_count=replica_count)

    def get_saver_class(self):
        from ..elastic_agent.ckpt_saver import CommonDirCheckpointSaver

        return CommonDirCheckpointSaver

    def load(self, resume_path="", target=None):
        """Memory first; then ``resume_path`` (this rank's persisted shard
        file -- shard layouts are framework-chosen, so there is no default
        file name to fall back to)."""
        step, sd = self.get_state_dict_from_memory(target=target)
        if sd:
            return sd
        if resume_path:
            return self._load_from_storage(resume_path, target)
        logger.warning(f"rank {self._rank}: no complete checkpoint in memory and no resume_path: nothing restored")
        return {}
