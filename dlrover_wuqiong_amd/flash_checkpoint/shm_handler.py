"""The flash-checkpoint shared-memory shard: header + payload + metadata.

Segment layout (one segment per local checkpoint shard)::

    [0, HEADER)        header: int64 words
                         0 magic, 1 payload bytes, 2 layout generation,
                         3 number of slices, 8+r  step of slice r complete
    [HEADER, ...)      payload: the coalesced tensor extents (layout.py)

A *slice* is a page-aligned sub-range of the payload written by one process:
for replicated (DDP) state every local rank writes 1/L of the payload in
parallel, each over its own PCIe link; for sharded state there is one slice.
A shard is complete for step ``s`` iff ``meta.config.step == s`` and every
slice word equals ``s`` (8-byte aligned stores: atomic on x86-64).

Metadata (tree of TensorMeta + CheckpointConfig) lives in a SharedDict so the
agent can rebuild the state dict after the worker is gone.

Parity: reference ``SharedMemoryHandler`` (``ckpt_saver.py:209-341``).
"""

import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import numpy as np

from ..common.log import logger
from ..common.multi_process import SharedDict, SharedMemory
from .layout import TensorMeta, tensors_from_payload

HEADER_BYTES = 64 * 1024
MAGIC = 0x44574B5053484D31  # "DWKPSHM1"
MAX_SLICES = 1024
DLROVER_CKPT_CONFIG_KEY = "_DLORVER_CKPT_CONFIG"
EVENT_QUEUE_SIZE = 16  # checkpoint events buffered between workers and the saver


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


class SharedMemoryHandler:
    def __init__(self, local_shard_id: int, host: bool = True):
        self.local_shard_id = local_shard_id
        self._shm_name = CheckpointSharedObjPrefix.SHM_NAME + str(local_shard_id)
        self.metadata = SharedDict(CheckpointSharedObjPrefix.META_NAME + str(local_shard_id), create=True)
        self.shared_memory: Optional[SharedMemory] = None
        self._header: Optional[np.ndarray] = None
        self._need_creation = True

    # ------------------------------------------------------------------ shm
    @property
    def shm_name(self):
        return self._shm_name

    def init_shared_memory(self, create: bool = False, size: int = 0) -> bool:
        """Create (payload ``size`` bytes) or attach the segment."""
        if self.shared_memory is not None:
            if not create or self.shared_memory.size == size + HEADER_BYTES:
                return True
            self.close()
        try:
            if create:
                self.shared_memory = SharedMemory(self._shm_name, create=True, size=size + HEADER_BYTES)
            else:
                self.shared_memory = SharedMemory(self._shm_name, create=False)
        except FileNotFoundError:
            self.shared_memory = None
            return False
        self._header = np.frombuffer(self.shared_memory.buf, dtype=np.int64, count=HEADER_BYTES // 8)
        if create:
            self._header[0] = MAGIC
            self._header[1] = size
        self._need_creation = False
        return True

    def exists(self) -> bool:
        return SharedMemory.exists(self._shm_name)

    @property
    def payload_addr(self) -> int:
        return self.shared_memory.addr + HEADER_BYTES

    @property
    def payload_size(self) -> int:
        return self.shared_memory.size - HEADER_BYTES if self.shared_memory else 0

    def payload_view(self):
        return self.shared_memory.buf[HEADER_BYTES:]

    # --------------------------------------------------------------- header
    def set_slice_step(self, idx: int, step: int):
        self._header[8 + idx] = step

    def slice_steps(self, n: int):
        if self._header is None:
            return []
        return [int(self._header[8 + i]) for i in range(n)]

    def reset_slices(self, n: int):
        if self._header is not None:
            self._header[8:8 + max(n, 1)] = 0

    # ------------------------------------------------------------- metadata
    def get_checkpoint_config(self, default_config: Optional[CheckpointConfig] = None) -> CheckpointConfig:
        meta = self.metadata.get()
        return meta.get(DLROVER_CKPT_CONFIG_KEY, default_config or CheckpointConfig())

    def set_metadata(self, meta_tree: Any, config: CheckpointConfig):
        d = {"tree": meta_tree, DLROVER_CKPT_CONFIG_KEY: config}
        self.metadata.set(d)

    def update_config(self, config: CheckpointConfig):
        d = self.metadata.get(local=True) or self.metadata.get()
        d[DLROVER_CKPT_CONFIG_KEY] = config
        self.metadata.set(d)

    def complete_step(self) -> int:
        """Step of the complete checkpoint in memory, 0 if none/partial."""
        meta = self.metadata.get()
        cfg: CheckpointConfig = meta.get(DLROVER_CKPT_CONFIG_KEY)
        if cfg is None or cfg.step <= 0:
            return 0
        if self.shared_memory is None or self._need_creation:
            if not self.init_shared_memory(create=False):
                return 0
        steps = self.slice_steps(cfg.num_slices)
        if steps and all(s == cfg.step for s in steps):
            return cfg.step
        return 0

    def no_checkpoint_state(self) -> bool:
        return self.complete_step() == 0

    no_checkpint_state = no_checkpoint_state  # reference spelling

    def load_state_dict(self) -> Dict:
        """Zero-copy CPU view of the complete checkpoint ({} if none)."""
        if self.complete_step() == 0:
            return {}
        meta = self.metadata.get()
        tree = meta.get("tree")
        if tree is None:
            return {}
        sd = tensors_from_payload(tree, self.shared_memory.buf, HEADER_BYTES)
        if isinstance(sd, dict):
            sd[DLROVER_CKPT_CONFIG_KEY] = meta.get(DLROVER_CKPT_CONFIG_KEY)
        return sd

    def reset(self):
        self._need_creation = True

    def close(self):
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
        self.metadata.unlink()
