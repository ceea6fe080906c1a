"""Pre-pinning of the node's flash-checkpoint shm before a worker needs it.

A restarted worker restores from the agent-owned shm segment.  The DMA
itself runs at ~55 GB/s per GPU, but the host range must first be
``hipHostRegister``'ed (page-table walk + pinning, ~0.5 s per 20 GB), and its
first save after the restart would pay the same for the other slot.  A deep
standby (``elastic_agent/standby.py``) calls
:func:`prepin_local_checkpoint_shm` while it waits: it maps the segment(s)
this local rank will touch, registers exactly its byte ranges (its slice of
every slot for a replicated checkpoint, the whole payload of its own shard
otherwise) with the process-wide :data:`~.copier.PINNED` registry, and parks
the mapping so the checkpoint engine adopts the *same* virtual addresses
(registrations are per address range).  Calling it again is cheap: a
segment that was re-created (new inode, e.g. resized) is unregistered,
unmapped and pinned afresh; ranges that became known later (slice metadata
written by the first save) are added.
"""

import time
from typing import Dict, List, Tuple

from ..common import env_utils
from ..common.log import logger
from ..common.multi_process import SharedDict, SharedMemory
from .shm_handler import (_ADOPTABLE, DLROVER_CKPT_CONFIG_KEY, HEADER_BYTES, MAGIC, CheckpointSharedObjPrefix,
                          adopt_mapping)

_PINNED_BYTES: Dict[str, int] = {}
_SLICE_BYTES: Dict[str, int] = {}  # segment -> this rank's slice bytes (layout known)
_STATE_BYTES: Dict[str, int] = {}  # segment -> its whole payload (the state the worker rebuilds)
_NSLICES: Dict[str, int] = {}  # segment -> slices of a replicated checkpoint (1: none)


def _slot_ranges(shm: SharedMemory, shard: int, local_rank: int,
                 nslices: Dict[str, int] = None) -> Tuple[List[Tuple[int, int]], bool]:
    """(addr, nbytes) of this rank's slice in every slot, and whether the
    slice layout is known (slot metadata written by a save)."""
    import numpy as np

    hdr = np.frombuffer(shm.buf, dtype=np.int64, count=HEADER_BYTES // 8)
    if int(hdr[0]) != MAGIC:
        return [], False
    size, stride, nslots = int(hdr[1]), int(hdr[3]), int(hdr[4])
    out = []
    known = False
    for s in range(nslots):
        try:
            meta = SharedDict(f"{CheckpointSharedObjPrefix.META_NAME}{shard}_{s}", create=False, timeout=0.2).get()
        except FileNotFoundError:
            meta = {}
        cfg = meta.get(DLROVER_CKPT_CONFIG_KEY)
        known = known or cfg is not None
        nsl = max(1, getattr(cfg, "num_slices", 1)) if cfg is not None else 1
        if cfg is not None and nslices is not None:
            nslices["nsl"] = nsl
        base = HEADER_BYTES + s * stride
        if nsl > 1:
            from .layout import split_ranges

            if local_rank >= nsl:
                continue
            lo, hi = split_ranges(size, nsl)[local_rank]
        elif shard == local_rank:
            lo, hi = 0, size
        else:
            continue
        if hi > lo:
            out.append((shm.addr + base + lo, hi - lo))
    return out, known


def prepinned_bytes() -> int:
    return sum(_PINNED_BYTES.values())


def local_state_bytes() -> int:
    """Payload bytes of the checkpoint this local rank restores (0: none yet):
    about the model + optimizer state its worker allocates."""
    return max(_STATE_BYTES.values(), default=0)


def local_slice_bytes() -> int:
    """Bytes of the payload slice this local rank snapshots (0: unknown yet)."""
    return max(_SLICE_BYTES.values(), default=0)


def restore_temp_bytes() -> int:
    """HBM of the replicated restore's all-gather temporary on this rank
    (``copier.restore``: world x per-round chunk; 0 without slices)."""
    from .hbm_budget import gather_chunk
    from .layout import split_ranges

    out = 0
    for name, nsl in _NSLICES.items():
        total = _STATE_BYTES.get(name, 0)
        if nsl > 1 and total > 0:
            per = split_ranges(total, nsl)[0][1]  # the padded slice every rank gathers (engine._restore_into)
            out = max(out, min(per, gather_chunk(per, nsl, free=1 << 62)) * nsl)
    return out


def prepin_local_checkpoint_shm() -> float:
    """Returns seconds spent.  No-op (0.0) when no segment exists yet."""
    import torch

    if not torch.cuda.is_available():
        return 0.0
    from .copier import PINNED

    t0 = time.time()
    lr = env_utils.get_local_rank()
    changed = False
    for shard in sorted({0, lr}):
        name = CheckpointSharedObjPrefix.SHM_NAME + str(shard)
        shm = _ADOPTABLE.get(name)
        if shm is not None and shm.stale():
            # re-created by the live workers (resize): drop the old pins + mapping
            PINNED.release_range(shm.addr, shm.size)
            _ADOPTABLE.pop(name, None)
            _PINNED_BYTES.pop(name, None)
            _SLICE_BYTES.pop(name, None)
            _STATE_BYTES.pop(name, None)
            _NSLICES.pop(name, None)
            shm.close()
            shm = None
        if shm is None:
            if not SharedMemory.exists(name):
                continue
            try:
                shm = SharedMemory(name, create=False)
            except FileNotFoundError:
                continue
        info: Dict[str, int] = {}
        ranges, known = _slot_ranges(shm, shard, lr, info)
        if known and ranges:
            _SLICE_BYTES[name] = ranges[0][1]
            _NSLICES[name] = info.get("nsl", 1)
            import numpy as np

            _STATE_BYTES[name] = int(np.frombuffer(shm.buf, dtype=np.int64, count=2)[1])
        if not ranges:
            if name not in _ADOPTABLE:
                shm.close()
            continue
        nbytes = 0
        for addr, n in ranges:
            # no explicit prefault: the live worker may be flushing into these
            # pages; hipHostRegister populates whatever is still missing
            if PINNED.covers(addr, n):
                nbytes += n
            elif PINNED.ensure(addr, n):
                nbytes += n
                changed = True
        adopt_mapping(name, shm)
        _PINNED_BYTES[name] = nbytes
    dt = time.time() - t0
    if changed:
        logger.info(f"standby pre-pinned checkpoint shm {dict(_PINNED_BYTES)} in {dt:.2f}s")
    return dt
