"""HBM budget of the flash-checkpoint data path on one GPU -- one place for
every sizing decision, so the checkpoint engine, the standbys and the tests
(mocked ``mem_get_info``, N=8 configurations) agree.

Per GPU (one rank per GPU; a replicated checkpoint is split 1/N across the
node's local ranks, a sharded one is already per rank):

* the live worker: model + optimizer state + activations (its peak);
* snapshot staging (``copier.py``): two full-slice buffers (double
  buffered: a save never waits for the previous flush), one, or a bounded
  ring of K chunks when not even one slice fits next to the worker;
* the HBM tier (``hbm_tier.py``): the staging buffers are owned by the
  standby and outlive the worker -- no extra bytes, same buffers;
* a deep standby: its own model + optimizer (it parks fully built);
  an import standby: only what it reserves in its caching allocator for
  the worker it will become (released under pressure, ``standby.py``);
* the replicated restore: the slice all-gather's temporary, bounded here
  to ``world x chunk`` (chunked gather) instead of the whole payload.

Reference: the reference sizes nothing on the device -- its snapshot is a
synchronous copy into pageable shm (``ckpt_saver.py:197-206``).
"""

import os
from dataclasses import asdict, dataclass, field
from typing import Dict, Optional

GiB = 1 << 30


def staging_reserve() -> int:
    """HBM kept free for the worker's own peaks when sizing staging buffers."""
    return int(os.environ.get("DWAMD_STAGING_RESERVE_GB", "24")) * GiB


def staging_buffers(free: int, have: int, nbytes: int, reserve: Optional[int] = None) -> int:
    """Full-slice staging buffers to keep: 2 when both fit next to the
    reserve (``have``: bytes this process already holds as staging)."""
    reserve = staging_reserve() if reserve is None else reserve
    return 2 if free + have >= 2 * nbytes + reserve else 1


def use_ring(free: int, have: int, nbytes: int, reserve: Optional[int] = None) -> bool:
    """Not even one full-slice buffer fits: snapshot through the bounded ring."""
    reserve = staging_reserve() if reserve is None else reserve
    return free + have < nbytes + reserve


def gather_chunk(per: int, world: int, free: int, cap: Optional[int] = None, margin: int = 4 * GiB) -> int:
    """Per-rank bytes per round of the restore all-gather: the whole slice
    (one round, temporary = world x per) when it fits in ``free - margin``
    and under ``cap`` (``DWAMD_RESTORE_GATHER_GB``, default 16 GiB total),
    else the largest 2 MiB multiple that does."""
    if per <= 0 or world <= 1:
        return per
    cap = int(float(os.environ.get("DWAMD_RESTORE_GATHER_GB", "16")) * GiB) if cap is None else cap
    room = max(0, min(cap, free - margin))
    if world * per <= room:
        return per
    c = room // world // (2 << 20) * (2 << 20)
    return max(64 << 20, c)


@dataclass
class HbmPlan:
    total: int
    worker_peak: int
    slice_bytes: int
    staging: str  # "double" | "single" | "ring"
    staging_bytes: int
    standby: str  # "deep" | "import"
    standby_bytes: int
    gather_chunk: int
    gather_temp_bytes: int
    restore_peak: int  # worker + staging + standby + the gather temporary
    fits: bool
    notes: Dict[str, str] = field(default_factory=dict)

    def as_dict(self) -> dict:
        d = asdict(self)
        for k in list(d):
            if k.endswith("bytes") or k in ("total", "worker_peak", "restore_peak", "gather_chunk"):
                d[k + "_gib"] = round(d.pop(k) / GiB, 2)
        return d


def plan(total: int, worker_state: int, worker_peak: int, payload: int, world_local: int, replicated: bool,
         standby: str = "import", ring_chunk: int = 1 << 30, ring_slots: int = 4,
         reserve: Optional[int] = None, import_reserve: bool = True) -> HbmPlan:
    """Decisions for ONE GPU of a node with ``world_local`` ranks.

    worker_state: model + optimizer bytes of a rank (what a deep standby
    also holds); worker_peak: the rank's peak footprint (state + activations);
    payload: the rank's checkpoint payload (the whole replicated state, or
    this rank's shard)."""
    notes = {}
    slice_bytes = -(-payload // world_local) if replicated else payload
    free_for_staging = total - worker_peak
    if standby == "deep":
        sb_bytes = worker_state
        if free_for_staging - sb_bytes < slice_bytes + (staging_reserve() if reserve is None else reserve):
            notes["standby"] = "deep standby does not fit next to the worker + one staging slice: import"
            standby, sb_bytes = "import", 0
    else:
        sb_bytes = 0
    free_for_staging -= sb_bytes
    if use_ring(free_for_staging, 0, slice_bytes, reserve):
        staging, st_bytes = "ring", min(ring_slots * ring_chunk, max(0, free_for_staging))
    elif staging_buffers(free_for_staging, 0, slice_bytes, reserve) == 2:
        staging, st_bytes = "double", 2 * slice_bytes
    else:
        staging, st_bytes = "single", slice_bytes
    if standby == "import" and import_reserve:
        # the import standby caches about the worker's peak, bounded by what
        # is left (it releases it when the worker's own use grows)
        sb_bytes = max(0, min(worker_peak, total - worker_peak - st_bytes - 8 * GiB))
    # restore: a NEW worker (after the failure the old one is gone) rebuilds
    # its state, then gathers; the standby's cache became that worker
    world_g = world_local if replicated else 1
    per = slice_bytes if replicated else payload
    free_at_restore = total - worker_state - st_bytes - (sb_bytes if standby == "deep" else 0)
    ch = gather_chunk(per, world_g, free_at_restore) if world_g > 1 else per
    temp = ch * world_g if world_g > 1 else 0
    if world_g > 1 and ch < per:
        notes["gather"] = f"restore gather chunked: {-(-per // ch)} rounds of {world_g} x {ch >> 20} MiB"
    steady = worker_peak + st_bytes + sb_bytes
    restore_peak = worker_state + st_bytes + (sb_bytes if standby == "deep" else 0) + temp
    return HbmPlan(total=total, worker_peak=worker_peak, slice_bytes=slice_bytes, staging=staging,
                   staging_bytes=st_bytes, standby=standby, standby_bytes=sb_bytes, gather_chunk=ch,
                   gather_temp_bytes=temp, restore_peak=restore_peak,
                   fits=steady <= total and restore_peak <= total, notes=notes)
