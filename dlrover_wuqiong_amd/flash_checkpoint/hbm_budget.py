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
* a deep standby: its own model + optimizer (it parks fully built) plus
  the rest of the worker's peak (activations) held in its caching
  allocator; an import standby: the worker's peak in its caching allocator
  (released under pressure, ``standby.py``).  With the HBM tier off the
  standby also holds its own staging buffers (``standby_staging``): the
  worker it becomes then allocates nothing on the restart path;
* the replicated restore: the slice all-gather's temporary, bounded here
  to ``world x chunk`` (chunked gather) instead of the whole payload, and
  reserved by the standby while it parks (``gather_temp_bytes``).

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
    else the largest 2 MiB multiple that does.  The restore itself passes
    an unbounded ``free``: the chunk is a collective size every rank must
    agree on (the standby reserved the temporary; the plan checks it fits)."""
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
    defer_steps: int  # ring staging: optimizer steps whose state write-back may be deferred (0: wait for the ring)
    defer_bytes: int  # HBM of the kept gradients of those steps
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
         reserve: Optional[int] = None, import_reserve: bool = True, hbm_tier: bool = True,
         grad_bytes: int = 0, staging_mode: str = "auto", ring_bytes: int = 0) -> HbmPlan:
    """Decisions for ONE GPU of a node with ``world_local`` ranks.

    worker_state: model + optimizer bytes of a rank (what a deep standby
    also holds); worker_peak: the rank's peak footprint (state + activations);
    payload: the rank's checkpoint payload (the whole replicated state, or
    this rank's shard); grad_bytes: the rank's gradient bytes (ring staging:
    a deferred optimizer-state write-back keeps one copy of the deferred
    elements' gradient per deferred step, optimizers/fused.py)."""
    notes = {}
    slice_bytes = -(-payload // world_local) if replicated else payload
    free_for_staging = total - worker_peak
    world_g = world_local if replicated else 1
    per = slice_bytes if replicated else payload
    # the restore all-gather temporary a standby reserves (sized like the
    # restore itself: copier.restore -> gather_chunk)
    temp_reserved = gather_chunk(per, world_g, 1 << 62) * world_g if world_g > 1 else 0
    if standby == "deep":
        sb_bytes = worker_peak + temp_reserved  # built state + activation peak + gather temporary
        if free_for_staging - sb_bytes < slice_bytes + (staging_reserve() if reserve is None else reserve):
            notes["standby"] = "deep standby does not fit next to the worker + one staging slice: import"
            standby, sb_bytes = "import", 0
    else:
        sb_bytes = 0
    free_for_staging -= sb_bytes
    if staging_mode == "ring" or (staging_mode != "full" and use_ring(free_for_staging, 0, slice_bytes, reserve)):
        # (copier._ring_shape: DWAMD_RING_HBM_GB when set, else K x C)
        staging, st_bytes = "ring", min(ring_bytes or ring_slots * ring_chunk, max(0, free_for_staging))
    elif staging_buffers(free_for_staging, 0, slice_bytes, reserve) == 2:
        staging, st_bytes = "double", 2 * slice_bytes
    else:
        staging, st_bytes = "single", slice_bytes
    defer_k, defer_b = 0, 0
    if staging == "ring" and grad_bytes > 0:
        kcap = max(1, min(7, int(os.environ.get("DWAMD_DEFER_STATE_STEPS", "4"))))
        # (the same 2 GiB margin as optimizers/fused.py _defer_budget)
        room = total - worker_peak - st_bytes - (sb_bytes if standby == "deep" else 0) - 2 * GiB
        defer_k = max(0, min(kcap, room // grad_bytes))
        defer_b = defer_k * grad_bytes
        notes["defer"] = (f"ring: state write-back deferred for up to {defer_k} steps ({defer_b / GiB:.1f} GiB of "
                          f"kept gradients)" if defer_k else "ring: no room for a kept gradient; steps wait for the ring")
    if standby == "import" and import_reserve:
        # the import standby caches about the worker's peak (+ the gather
        # temporary), bounded by what is left (it releases it when the
        # worker's own use grows); with the tier off it also holds its own
        # staging buffers next to the live worker's
        own_staging = 0 if (hbm_tier or staging == "ring") else st_bytes
        sb_bytes = max(0, min(worker_peak + temp_reserved,
                              total - worker_peak - st_bytes - own_staging - defer_b - 8 * GiB))
        sb_bytes += own_staging
    # restore: a NEW worker (after the failure the old one is gone) rebuilds
    # its state, then gathers into the temporary its standby reserved
    free_at_restore = total - worker_state - st_bytes - (sb_bytes if standby == "deep" else 0)
    ch = gather_chunk(per, world_g, free_at_restore + temp_reserved) if world_g > 1 else per
    temp = ch * world_g if world_g > 1 else 0
    if world_g > 1 and ch < per:
        notes["gather"] = f"restore gather chunked: {-(-per // ch)} rounds of {world_g} x {ch >> 20} MiB"
    steady = worker_peak + st_bytes + sb_bytes + defer_b
    # the recovered worker holds what its standby held (the temporary inside it)
    restore_peak = max(worker_state + temp, sb_bytes) + st_bytes + (sb_bytes if standby == "deep" else 0)
    return HbmPlan(total=total, worker_peak=worker_peak, slice_bytes=slice_bytes, staging=staging,
                   staging_bytes=st_bytes, standby=standby, standby_bytes=sb_bytes, gather_chunk=ch,
                   gather_temp_bytes=temp, restore_peak=restore_peak, defer_steps=defer_k, defer_bytes=defer_b,
                   fits=steady <= total and restore_peak <= total, notes=notes)


# ------------------------------------------------------------------ host side
class HostMemoryError(RuntimeError):
    """The node's host memory cannot hold even one checkpoint slot."""


def read_meminfo(path: str = "/proc/meminfo") -> Dict[str, int]:
    out = {}
    try:
        with open(path) as f:
            for line in f:
                k, _, v = line.partition(":")
                parts = v.split()
                if parts:
                    out[k.strip()] = int(parts[0]) * (1024 if len(parts) > 1 and parts[1] == "kB" else 1)
    except OSError:
        pass
    return out


def shm_free_bytes(path: str = "/dev/shm") -> int:
    try:
        st = os.statvfs(path)
        return st.f_bavail * st.f_frsize
    except OSError:
        return 0


def host_reserve(mem_total: int) -> int:
    """Host RAM kept for everything that is not checkpoint shm (the
    processes' own memory, page cache for data loading, pinned staging)."""
    gb = os.environ.get("DWAMD_HOST_RESERVE_GB")
    return int(float(gb) * GiB) if gb else max(8 * GiB, mem_total // 20)


@dataclass
class HostPlan:
    segments: int  # checkpoint segments on this node (1 replicated, one per local shard otherwise)
    slot_bytes: int  # per segment per slot (aligned payload)
    slots: int  # 2 (double-buffered: a save never overwrites the latest checkpoint), 1, or 0 = does not fit
    need_bytes: int  # segments x (header + slots x slot_bytes)
    shm_free: int
    mem_available: int
    reclaimable: int  # bytes of this job's existing segments (replaced by the new ones)
    reserve: int
    room: int
    pin_sec_est: float  # first-save prefault + hipHostRegister of one segment at DWAMD_PIN_GBPS
    fits: bool
    notes: Dict[str, str] = field(default_factory=dict)

    def as_dict(self) -> dict:
        d = asdict(self)
        for k in list(d):
            if k.endswith("bytes") or k in ("shm_free", "mem_available", "reclaimable", "reserve", "room"):
                d[k + "_gib"] = round(d.pop(k) / GiB, 2)
        return d


def host_plan(payload: int, segments: int, want_slots: int = 2, shm_free: Optional[int] = None,
              meminfo: Optional[Dict[str, int]] = None, reclaimable: int = 0,
              reserve: Optional[int] = None, pin_gbps: Optional[float] = None) -> HostPlan:
    """Node-level host memory plan of the flash-checkpoint shm (tmpfs).

    tmpfs over-commits: a segment is created at any size and its pages are
    allocated on first touch, so an undersized node dies with SIGBUS in the
    middle of a snapshot flush instead of failing cleanly.  Sized here
    before any segment exists: room = min(free /dev/shm, MemAvailable -
    reserve) + this job's segments that the new ones replace.  Two slots
    when they fit, one (with a warning: a crash during a save then loses the
    in-memory checkpoint) when only one does, else :class:`HostMemoryError`.

    Reference: ``ckpt_saver.py:140`` ``_create_shared_memory`` creates the
    segment unconditionally."""
    from .shm_handler import HEADER_BYTES, SLOT_ALIGN

    mi = read_meminfo() if meminfo is None else meminfo
    shm_free = shm_free_bytes() if shm_free is None else shm_free
    mem_avail = mi.get("MemAvailable", 0)
    reserve = host_reserve(mi.get("MemTotal", 0)) if reserve is None else reserve
    slot = (payload + SLOT_ALIGN - 1) // SLOT_ALIGN * SLOT_ALIGN
    room = max(0, min(shm_free, mem_avail - reserve)) + reclaimable
    notes = {}
    slots = 0
    for s in range(max(1, want_slots), 0, -1):
        if segments * (HEADER_BYTES + s * slot) <= room:
            slots = s
            break
    if 0 < slots < want_slots:
        notes["slots"] = (f"{want_slots} slots need {segments * want_slots * slot / GiB:.1f} GiB of host shm, "
                          f"{room / GiB:.1f} GiB available: {slots} slot (a failure during a save loses the "
                          f"in-memory checkpoint; storage is the fallback)")
    elif slots == 0:
        notes["slots"] = (f"one slot needs {segments * slot / GiB:.1f} GiB of host shm, only {room / GiB:.1f} GiB "
                          f"available (/dev/shm free {shm_free / GiB:.1f}, MemAvailable {mem_avail / GiB:.1f}, "
                          f"reserve {reserve / GiB:.1f})")
    rate = float(os.environ.get("DWAMD_PIN_GBPS", "2.7")) if pin_gbps is None else pin_gbps
    n_slots = max(slots, 1)
    return HostPlan(segments=segments, slot_bytes=slot, slots=slots,
                    need_bytes=segments * (HEADER_BYTES + n_slots * slot), shm_free=shm_free,
                    mem_available=mem_avail, reclaimable=reclaimable, reserve=reserve, room=room,
                    pin_sec_est=round(n_slots * slot / (rate * 1e9), 2) if rate > 0 else 0.0,
                    fits=slots > 0, notes=notes)
