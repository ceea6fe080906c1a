"""The flash-checkpoint shared-memory shard: header + double-buffered payload.

Segment layout (one segment per local checkpoint shard)::

    [0, HEADER)                   header: int64 words
                                    0 magic, 1 payload bytes (per slot),
                                    2 layout generation, 3 slot stride,
                                    4 number of slots, 5 owner (hash of the
                                    writing job's checkpoint dir, 0 = any),
                                    8 + s*MAX_SLICES + r: step of slice r of slot s
                                    META_WORDS + 2s, +1: step / slice count of
                                      slot s's metadata (read without unpickling it)
    [HEADER + s*stride, ...)      payload slot s: the coalesced tensor extents

Two payload *slots*: a save always writes the slot that does NOT hold the
latest complete checkpoint, so a process that dies in the middle of a
snapshot/flush (the D2H flush of a 1.5B-parameter state takes ~0.4 s, i.e.
a large fraction of a short checkpoint interval) still leaves the previous
complete checkpoint intact in memory, and the agent can persist slot A while
training already snapshots into slot B.  (The reference keeps one buffer:
a crash during a save loses the in-memory checkpoint.)  ``DWAMD_CKPT_SLOTS=1``
restores the single-buffer behaviour to halve host memory.

A *slice* is a page-aligned sub-range of the payload written by one process:
for replicated (DDP) state every local rank writes 1/L of the payload in
parallel, each over its own PCIe link; for sharded state there is one slice.
Slot ``s`` is complete for step ``t`` iff its metadata config has
``step == t`` and every slice word of the slot equals ``t`` (8-byte aligned
stores: atomic on x86-64).  A writer zeroes its slice word before touching
the slot's bytes, so a partially written slot never reads as complete.

Metadata (tree of TensorMeta + CheckpointConfig) lives in one SharedDict per
slot so the agent can rebuild the state dict after the worker is gone.

Parity: reference ``SharedMemoryHandler`` (``ckpt_saver.py:209-341``).
"""

import os
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import numpy as np

from ..common.log import logger
from ..common.multi_process import SharedDict, SharedMemory
from .layout import TensorMeta, tensors_from_payload  # noqa: F401  (TensorMeta re-exported)

HEADER_BYTES = 64 * 1024
MAGIC = 0x44574B5053484D32  # "DWKPSHM2"
MAX_SLICES = 1024
SLOT_ALIGN = 2 << 20
META_WORDS = 7168  # header word index of slot 0's (metadata step, num_slices)
OWNER_WORD = 5
DLROVER_CKPT_CONFIG_KEY = "_DLORVER_CKPT_CONFIG"
EVENT_QUEUE_SIZE = 16  # checkpoint events buffered between workers and the saver


_ADOPTABLE: Dict[str, SharedMemory] = {}


def adopt_mapping(name: str, shm: SharedMemory):
    """Park an already-mapped (and typically hipHostRegister'ed) segment so
    the next attach of ``name`` in this process reuses the same addresses
    (see ``prewarm.py``)."""
    _ADOPTABLE[name] = shm


def _open_segment(name: str) -> SharedMemory:
    shm = _ADOPTABLE.pop(name, None)
    if shm is not None and not shm.stale() and not shm._closed:
        return shm
    return SharedMemory(name, create=False)


def default_num_slots() -> int:
    return max(1, min(2, int(os.environ.get("DWAMD_CKPT_SLOTS", "2"))))


class CheckpointSharedObjPrefix:
    SAVE_STEP_QNAME = "checkpoint_lock_rank_"
    META_NAME = "checkpoint_meta_"
    SHM_NAME = "checkpoint_shm_"
    SHM_LOCK_NAME = "shm_lock_"


@dataclass
class CheckpointConfig:
    """Reference ``ckpt_saver.py:CheckpointConfig`` (+ slice bookkeeping)."""

    rank: int = 0
    group_rank: int = 0
    world_size: int = 0
    step: int = 0
    writing_shm: bool = False
    paths: Dict[str, str] = field(default_factory=dict)
    num_slices: int = 1
    generation: int = 0


def slot_lock_name(local_shard_id: int, slot: int) -> str:
    return f"{CheckpointSharedObjPrefix.SHM_LOCK_NAME}{local_shard_id}_{slot}"


class SharedMemoryHandler:
    def __init__(self, local_shard_id: int, host: bool = True, num_slots: Optional[int] = None):
        self.local_shard_id = local_shard_id
        # capacity (metadata dicts / slot locks exist for this many slots);
        # ``num_slots`` is the segment's active count: the host-memory plan
        # may create it with fewer (hbm_budget.host_plan), readers adopt the
        # count from the segment header
        self.max_slots = num_slots or default_num_slots()
        self.num_slots = self.max_slots
        self._shm_name = CheckpointSharedObjPrefix.SHM_NAME + str(local_shard_id)
        self.metas = [SharedDict(f"{CheckpointSharedObjPrefix.META_NAME}{local_shard_id}_{s}", create=True)
                      for s in range(self.num_slots)]
        self.shared_memory: Optional[SharedMemory] = None
        self._header: Optional[np.ndarray] = None
        self._need_creation = True
        self.before_unmap: Optional[Callable[[], None]] = None

    # ------------------------------------------------------------------ shm
    @property
    def shm_name(self):
        return self._shm_name

    @staticmethod
    def _stride(size: int) -> int:
        return (size + SLOT_ALIGN - 1) // SLOT_ALIGN * SLOT_ALIGN

    def init_shared_memory(self, create: bool = False, size: int = 0, owner: int = 0,
                           slots: Optional[int] = None) -> bool:
        """Create (``size`` payload bytes per slot) or attach the segment.
        ``owner`` (create only): the writing job's id; a segment another job
        wrote is re-created instead of reused (its steps are not ours).
        ``slots`` (create only): active slot count of a new segment (<=
        ``max_slots``; default all)."""
        if self.shared_memory is not None and self.shared_memory.stale():
            self.close()  # re-created by a writer (resize): drop the old mapping
        if self.shared_memory is not None:
            if not create or (self._header is not None and int(self._header[1]) == size
                              and self._owned_by(owner)):
                return True
            self.close()
        if create and self.init_shared_memory(create=False) and int(self._header[1]) == size \
                and self._owned_by(owner):
            if owner:
                self._header[OWNER_WORD] = owner
            return True  # compatible segment (e.g. from before a restart): keep its checkpoints
        self.close()
        try:
            if create:
                if self.exists():
                    # never resize in place: a reader's mapping could fault (SIGBUS)
                    SharedMemory(self._shm_name, create=False).unlink()
                stride = self._stride(size)
                self.num_slots = max(1, min(self.max_slots, slots or self.max_slots))
                self.shared_memory = SharedMemory(self._shm_name, create=True,
                                                  size=HEADER_BYTES + stride * self.num_slots)
            else:
                self.shared_memory = _open_segment(self._shm_name)
        except FileNotFoundError:
            self.shared_memory = None
            return False
        self._header = np.frombuffer(self.shared_memory.buf, dtype=np.int64, count=HEADER_BYTES // 8)
        if create:
            self._header[8:] = 0
            self._header[0] = MAGIC
            self._header[1] = size
            self._header[3] = self._stride(size)
            self._header[4] = self.num_slots
            self._header[OWNER_WORD] = owner
            for m in self.metas:
                m.set({})
        elif int(self._header[0]) != MAGIC or not 1 <= int(self._header[4]) <= self.max_slots:
            logger.warning(f"shm {self._shm_name}: incompatible header; ignoring it")
            self.close()
            return False
        else:
            self.num_slots = int(self._header[4])  # the creator's (host-memory plan) decision
        self._need_creation = False
        return True

    def _owned_by(self, owner: int) -> bool:
        return not owner or self._header is None or int(self._header[OWNER_WORD]) in (0, owner)

    def owner(self) -> int:
        return int(self._header[OWNER_WORD]) if self._header is not None else 0

    def exists(self) -> bool:
        return SharedMemory.exists(self._shm_name)

    def payload_addr(self, slot: int = 0) -> int:
        return self.shared_memory.addr + self.payload_offset(slot)

    def payload_offset(self, slot: int = 0) -> int:
        return HEADER_BYTES + slot * int(self._header[3])

    @property
    def payload_size(self) -> int:
        return int(self._header[1]) if self.shared_memory is not None and self._header is not None else 0

    def payload_view(self, slot: int = 0):
        off = self.payload_offset(slot)
        return self.shared_memory.buf[off: off + self.payload_size]

    # --------------------------------------------------------------- header
    def set_slice_step(self, slot: int, idx: int, step: int):
        self._header[8 + slot * MAX_SLICES + idx] = step

    def slice_steps(self, slot: int, n: int) -> List[int]:
        if self._header is None:
            return []
        base = 8 + slot * MAX_SLICES
        return [int(self._header[base + i]) for i in range(n)]

    # HBM-tier stamps (see hbm_tier.py): (step, owner pid, nbytes) per
    # (slice, staging buffer)
    def set_hbm_stamp(self, slice_idx: int, buf: int, step: int, pid: int = 0, nbytes: int = 0):
        from .hbm_tier import MAX_STAMP_SLICES, stamp_index

        if self._header is None or slice_idx >= MAX_STAMP_SLICES:
            return
        i = stamp_index(slice_idx, buf)
        if step == 0:
            self._header[i] = 0  # invalidate first: a reader never sees a stale step with new bytes
            self._header[i + 1] = 0
            self._header[i + 2] = 0
        else:
            self._header[i + 1] = pid
            self._header[i + 2] = nbytes
            self._header[i] = step

    def hbm_stamp(self, slice_idx: int, buf: int):
        from .hbm_tier import MAX_STAMP_SLICES, stamp_index

        if self._header is None or slice_idx >= MAX_STAMP_SLICES:
            return 0, 0, 0
        i = stamp_index(slice_idx, buf)
        return int(self._header[i]), int(self._header[i + 1]), int(self._header[i + 2])

    def reset_slices(self, slot: int, n: int):
        if self._header is not None:
            base = 8 + slot * MAX_SLICES
            self._header[base: base + max(n, 1)] = 0

    # ------------------------------------------------------------- metadata
    def get_meta(self, slot: int) -> dict:
        return self.metas[slot].get() or {}

    def get_checkpoint_config(self, default_config: Optional[CheckpointConfig] = None,
                              slot: Optional[int] = None) -> CheckpointConfig:
        if slot is None:
            slot = self.latest_slot()
        if slot < 0:
            return default_config or CheckpointConfig()
        return self.get_meta(slot).get(DLROVER_CKPT_CONFIG_KEY, default_config or CheckpointConfig())

    def set_metadata(self, slot: int, meta_tree: Any, config: CheckpointConfig):
        self.set_meta_dict(slot, {"tree": meta_tree, DLROVER_CKPT_CONFIG_KEY: config})

    def set_meta_dict(self, slot: int, meta: dict):
        """Write a slot's metadata: the pickled dict, then its (step, slice
        count) header words -- what completeness checks read."""
        cfg = meta.get(DLROVER_CKPT_CONFIG_KEY)
        if self._header is not None:
            self._header[META_WORDS + 2 * slot] = 0
        self.metas[slot].set(meta)
        if self._header is not None and cfg is not None:
            self._header[META_WORDS + 2 * slot + 1] = max(1, int(cfg.num_slices))
            self._header[META_WORDS + 2 * slot] = int(cfg.step)

    def _attached(self) -> bool:
        if self.shared_memory is not None and not self.shared_memory.stale():
            self._need_creation = False
            return True
        self.close()
        return self.init_shared_memory(create=False)

    def slot_step(self, slot: int) -> int:
        """Step of the complete checkpoint in ``slot``; 0 if none/partial.
        Reads header words only (a save checks both slots: unpickling the
        metadata trees would cost milliseconds of training pause)."""
        if not self._attached() or self._header is None:
            return 0
        step = int(self._header[META_WORDS + 2 * slot])
        if step <= 0:
            return 0
        steps = self.slice_steps(slot, int(self._header[META_WORDS + 2 * slot + 1]))
        if steps and all(s == step for s in steps):
            return step
        return 0

    def complete_steps(self) -> Dict[int, int]:
        """{step: slot} of every complete in-memory checkpoint."""
        out = {}
        for s in range(self.num_slots):
            st = self.slot_step(s)
            if st > 0:
                out[st] = s
        return out

    def complete_step(self) -> int:
        """Step of the latest complete checkpoint in memory, 0 if none."""
        steps = self.complete_steps()
        return max(steps) if steps else 0

    def latest_slot(self) -> int:
        steps = self.complete_steps()
        return steps[max(steps)] if steps else -1

    def slot_of(self, step: int) -> int:
        return self.complete_steps().get(step, -1)

    def write_slot(self) -> int:
        """The slot the next save writes: never the latest complete one."""
        latest = self.latest_slot()
        if latest < 0:
            return 0
        return (latest + 1) % self.num_slots

    def no_checkpoint_state(self) -> bool:
        return self.complete_step() == 0

    no_checkpint_state = no_checkpoint_state  # reference spelling

    def load_state_dict(self, slot: Optional[int] = None) -> Dict:
        """Zero-copy CPU view of a complete checkpoint ({} if none)."""
        if slot is None:
            slot = self.latest_slot()
        if slot < 0 or self.slot_step(slot) == 0:
            return {}
        meta = self.get_meta(slot)
        tree = meta.get("tree")
        if tree is None:
            return {}
        sd = tensors_from_payload(tree, self.shared_memory.buf, self.payload_offset(slot))
        if isinstance(sd, dict):
            sd[DLROVER_CKPT_CONFIG_KEY] = meta.get(DLROVER_CKPT_CONFIG_KEY)
        return sd

    # ---------------------------------------------------- replica transport
    def export_slot(self, slot: int):
        """(payload bytes view, metadata) of a complete slot, for replicas."""
        return self.payload_view(slot), self.get_meta(slot)

    def import_slot(self, data, meta: dict):
        """Install a peer's copy as this shard's (only) complete checkpoint."""
        self.close()
        self.init_shared_memory(create=True, size=len(data))
        off = self.payload_offset(0)
        self.shared_memory.buf[off: off + len(data)] = data
        cfg: CheckpointConfig = meta[DLROVER_CKPT_CONFIG_KEY]
        self.set_meta_dict(0, meta)
        for r in range(cfg.num_slices):
            self.set_slice_step(0, r, cfg.step)

    def reset(self):
        self._need_creation = True

    def close(self):
        if self.shared_memory is not None and self.before_unmap is not None:
            # the owner's background users of this mapping (prefault/pin
            # thread, in-flight D2H flushes) must finish before it goes away
            self.before_unmap()
        self._header = None
        if self.shared_memory is not None:
            try:
                self.shared_memory.close()
            except Exception:
                pass
            self.shared_memory = None

    def unlink(self):
        try:
            if self.shared_memory is None:
                self.init_shared_memory(create=False)
            if self.shared_memory is not None:
                self.shared_memory.unlink()
        except Exception as e:  # pragma: no cover
            logger.warning(f"unlink shm {self._shm_name}: {e}")
        self.close()
        for m in self.metas:
            m.unlink()
