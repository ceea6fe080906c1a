"""Byte movement between live tensors and the shm payload.

GPU save path (what the training loop pays for):
  1. ONE ``dw_multi_copy`` launch on the compute stream snapshots this
     process's payload slice (HBM -> HBM staging buffer, 16-byte vector
     streams, all 256 CUs).  Training may mutate parameters right after: the
     snapshot is ordered before them on the same stream.
  2. A background thread makes a side HIP stream wait on the snapshot event
     and issues ``hipMemcpyAsync`` staging -> *pinned* shm (the segment is
     registered with ``hipHostRegister``), then stamps the slice step in the
     shm header.  PCIe time is hidden behind the next training steps.

GPU load path: H2D of this process's slice from pinned shm, then (for a
replicated checkpoint split across the node's local ranks) an RCCL
``all_gather_into_tensor`` over xGMI re-assembles the full payload on every
GPU, and ONE ``dw_multi_copy`` scatters it into the live tensors.

Reference behaviour being replaced: per-tensor synchronous
``torch.frombuffer(...).copy_(gpu_tensor)`` into pageable memory
(``ckpt_saver.py:197-206``) and per-tensor H2D on load.
"""

import ctypes
import os
import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch

from ..common.log import logger
from .._native import runtime
from .layout import Extent, Layout, TensorMeta, intersect_extents, iter_leaves

CHUNK = 1 << 20  # descriptor granularity for the multi-copy kernel


def _kern():
    from .._native import kernels

    return kernels(required=True)


def _check(err, what):
    if err != 0:
        msg = _kern().dw_hip_error_string(err)
        raise RuntimeError(f"{what}: hip error {err} ({msg.decode() if msg else ''})")


def build_descs(pieces: List[Tuple[int, int, int]], device) -> torch.Tensor:
    """pieces: (src_addr, dst_addr, nbytes) -> device int64 [n, 3] chunked."""
    parts = []
    for s, d, n in pieces:
        if n <= 0:
            continue
        o = np.arange(0, n, CHUNK, dtype=np.uint64)  # vectorised: a 22 GB restore is ~21k rows
        blk = np.empty((o.size, 3), dtype=np.uint64)
        blk[:, 0] = o + np.uint64(s)
        blk[:, 1] = o + np.uint64(d)
        blk[:, 2] = np.minimum(np.uint64(CHUNK), np.uint64(n) - o)
        parts.append(blk)
    if not parts:
        return torch.empty(0, 3, dtype=torch.int64, device=device)
    arr = (parts[0] if len(parts) == 1 else np.concatenate(parts)).view(np.int64)
    return torch.from_numpy(arr).to(device, non_blocking=False)


def launch_multi_copy(descs: torch.Tensor, stream=None, max_blocks: int = 0):
    if descs.numel() == 0:
        return
    s = stream if stream is not None else torch.cuda.current_stream()
    _check(_kern().dw_multi_copy_grid(ctypes.c_void_p(descs.data_ptr()), descs.shape[0], int(max_blocks),
                                      ctypes.c_void_p(s.cuda_stream)), "multi_copy")


class PrepTracker:
    """Futures of the background prefault + registration of shm ranges
    (engine ``_start_shm_prep``): a flush waits only for the ranges it
    writes, so the first save of a fresh segment never waits for the other
    slot's preparation."""

    def __init__(self):
        self._ranges: List[Tuple[int, int, Future]] = []

    def add(self, addr: int, nbytes: int) -> Future:
        f: Future = Future()
        self._ranges.append((addr, addr + nbytes, f))
        return f

    def wait(self, addr: Optional[int] = None, nbytes: int = 0):
        for a, e, f in self._ranges:
            if addr is None or (a < addr + nbytes and addr < e):
                f.result()

    result = wait  # Future-like: wait for everything

    def fail_pending(self):
        for _a, _e, f in self._ranges:
            if not f.done():
                f.set_result(None)


class PinnedRegistry:
    """Tracks hipHostRegister'ed ranges of shm mappings."""

    def __init__(self):
        self._ranges: List[Tuple[int, int]] = []
        self._lock = threading.Lock()
        self.piece = max(64, int(os.environ.get("DWAMD_PREP_PIECE_MB", "1024"))) << 20

    def ensure(self, addr: int, nbytes: int) -> bool:
        if nbytes <= 0:
            return True
        page = 4096
        a = addr // page * page
        e = (addr + nbytes + page - 1) // page * page
        with self._lock:
            # register only the parts of [a, e) not yet covered
            gaps, cur = [], a
            for (ra, re) in sorted(self._ranges):
                if re <= cur or ra >= e:
                    continue
                if ra > cur:
                    gaps.append((cur, ra))
                cur = max(cur, re)
                if cur >= e:
                    break
            if cur < e:
                gaps.append((cur, e))
        # register in pieces, the lock released in between: one huge
        # hipHostRegister holds the process's mm lock (and the runtime's) for
        # seconds, stalling the training thread's allocations and launches
        for ga, ge in gaps:
            o = ga
            while o < ge:
                with self._lock:  # another thread may have registered parts meanwhile
                    inside = next((re for ra, re in self._ranges if ra <= o < re), None)
                    if inside is not None:
                        o = inside
                        continue
                    nxt = min([ra for ra, _re in self._ranges if ra > o] + [ge])
                    c = min(self.piece, nxt - o)
                    err = _kern().dw_host_register(ctypes.c_void_p(o), c)
                    if err != 0:
                        logger.warning(f"hipHostRegister({c} B) failed with {err}; using pageable copies")
                        return False
                    self._ranges.append((o, o + c))
                o += c
        return True

    def split(self, addr: int, nbytes: int) -> List[Tuple[int, int, bool]]:
        """Cut [addr, addr+nbytes) at registration boundaries: HIP rejects a
        pinned-kind copy whose host range spans two hipHostRegister'ed
        allocations ("invalid argument").  Returns (addr, n, pinned)."""
        end = addr + nbytes
        out: List[Tuple[int, int, bool]] = []
        cur = addr
        with self._lock:
            ranges = sorted(self._ranges)
        for ra, re in ranges:
            if re <= cur:
                continue
            if ra >= end:
                break
            if ra > cur:
                out.append((cur, ra - cur, False))
                cur = ra
            e = min(re, end)
            out.append((cur, e - cur, True))
            cur = e
            if cur >= end:
                break
        if cur < end:
            out.append((cur, end - cur, False))
        return out

    def release_all(self):
        with self._lock:
            for (a, _e) in self._ranges:
                _kern().dw_host_unregister(ctypes.c_void_p(a))
            self._ranges.clear()

    def release_range(self, addr: int, nbytes: int):
        """Unregister every registration that lies inside [addr, addr+nbytes)
        (a mapping that is about to be unmapped)."""
        end = addr + nbytes
        with self._lock:
            keep = []
            for (a, e) in self._ranges:
                if a >= addr and e <= end:
                    _kern().dw_host_unregister(ctypes.c_void_p(a))
                else:
                    keep.append((a, e))
            self._ranges = keep

    def covers(self, addr: int, nbytes: int) -> bool:
        return all(p for _a, _n, p in self.split(addr, nbytes))


# One registry per process: a deep standby pre-registers the checkpoint shm
# (prewarm.py) before the engine and its copier exist.
PINNED = PinnedRegistry()


_FENCED = None  # copiers with a pending overlapped snapshot (weak set)
_OPTIMIZERS = None  # optimizers seen stepping (weak set): their tensors are written only in step()


def _optimizer_step_fence(opt, _args, _kwargs):
    _OPTIMIZERS.add(opt)
    offer = getattr(opt, "offer_ring_fence", None)
    for c in list(_FENCED):
        # a pending RING snapshot: an optimizer that can defer the write-back
        # of its not-yet-copied state (optimizers/fused.py) takes the fence
        # over instead of stalling its update until the ring has drained
        if offer is not None and c.ring_pending() and offer(c):
            continue
        c.fence()
        _FENCED.discard(c)


_FLUSH_STREAMS: dict = {}  # device index -> a flush stream created early (precreate_flush_stream)


def precreate_flush_stream(device) -> torch.cuda.Stream:
    """Create this device's checkpoint flush stream now (the next copier of
    this process adopts it): hardware queues are assigned in creation order
    (see elastic_agent/standby.py)."""
    idx = torch.device(device).index or 0
    if idx not in _FLUSH_STREAMS:
        _FLUSH_STREAMS[idx] = torch.cuda.Stream(device=device)
    return _FLUSH_STREAMS[idx]


def _snapshot_stream(device) -> torch.cuda.Stream:
    """The stream of overlapped / ring snapshot copies: HIGH priority.  HIP
    shares hardware queues among the streams of one priority once a process
    has more than GPU_MAX_HW_QUEUES of them; a snapshot copy queued behind the
    previous checkpoint's 0.4 s PCIe flush (normal priority) stalled the next
    optimizer step's fence by that much (GPT2-1.5B, overlapped snapshots:
    steps after a save 491 ms).  A different priority is a different queue."""
    try:
        return torch.cuda.Stream(device=device, priority=-1)
    except Exception:
        return torch.cuda.Stream(device=device)


def _merge(ranges: List[Tuple[int, int]]) -> List[Tuple[int, int]]:
    out: List[Tuple[int, int]] = []
    for a, b in sorted(r for r in ranges if r[1] > r[0]):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def register_optimizer(opt):
    """Declare an optimizer whose parameters/state are written only inside
    its ``step()`` (done automatically at its first step)."""
    _install_fence_hook()
    _OPTIMIZERS.add(opt)


def fence_all():
    """Order the current stream after every pending overlapped snapshot: call
    before writing checkpointed tensors outside ``Optimizer.step`` (e.g. a
    SAM first step)."""
    if _FENCED:
        for c in list(_FENCED):
            c.fence()
        _FENCED.clear()


def _step_only_ranges() -> List[Tuple[int, int]]:
    """Sorted, merged device address ranges of every storage that only an
    optimizer step writes (parameters + optimizer state of the optimizers
    seen so far).  An overlapped snapshot may read these after the save call
    returns; anything else (BatchNorm running stats, EMA buffers, ...) can be
    written by the next forward and is copied before the call returns."""
    rng = []
    for opt in list(_OPTIMIZERS or ()):
        ts = [p for g in opt.param_groups for p in g["params"]]
        for st in opt.state.values():
            ts.extend(v for v in st.values() if torch.is_tensor(v))
        extra = getattr(opt, "checkpoint_safe_tensors", None)
        if extra is not None:
            ts.extend(extra())
        for t in ts:
            t = getattr(t, "_local_tensor", t)
            if t is None or not t.is_cuda:
                continue
            s = t.untyped_storage()
            if s.nbytes():
                rng.append((s.data_ptr(), s.data_ptr() + s.nbytes()))
    rng.sort()
    merged: List[Tuple[int, int]] = []
    for a, b in rng:
        if merged and a <= merged[-1][1]:
            merged[-1] = (merged[-1][0], max(merged[-1][1], b))
        else:
            merged.append((a, b))
    return merged


def _covered(ranges: List[Tuple[int, int]], starts: List[int], a: int, n: int) -> bool:
    import bisect

    i = bisect.bisect_right(starts, a) - 1
    return i >= 0 and a + n <= ranges[i][1]


def _pending_updates(device) -> list:
    """Events of optimizer updates still running on a side stream
    (``optimizers/overlap.py``): a snapshot must read after them."""
    from ..optimizers.overlap import pending_events
    from . import deferred_restore

    # ... and optimizer state a restart's restore is still copying in
    return pending_events(device) + deferred_restore.events(device)


def _flush_deferred_state():
    """Optimizers that deferred the write-back of state a ring snapshot was
    still copying (optimizers/fused.py) complete it before anything
    snapshots that state again."""
    from ..optimizers.fused import flush_deferred_state

    flush_deferred_state()


def device_free_bytes(device) -> int:
    """HBM a new allocation of this process can get without growing its
    footprint: the driver's free memory plus what the caching allocator
    holds unused (a standby's reservation the worker grows into)."""
    free, _total = torch.cuda.mem_get_info(device)
    try:
        cached = torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)
    except Exception:
        cached = 0
    return int(free) + max(0, int(cached))


def _install_fence_hook():
    global _FENCED, _OPTIMIZERS
    if _FENCED is None:
        import weakref

        from torch.optim.optimizer import register_optimizer_step_pre_hook

        _FENCED = weakref.WeakSet()
        _OPTIMIZERS = weakref.WeakSet()
        register_optimizer_step_pre_hook(_optimizer_step_fence)


class GpuCopier:
    """Per-process GPU <-> shm mover with a persistent staging buffer."""

    def __init__(self, device: torch.device, flush_cu_stride: Optional[int] = None):
        import os

        self.device = device
        # The runtime implements D2H/H2D to pinned host memory with blit
        # kernels; on a plain stream one 20 GB flush occupies every CU for
        # ~0.4 s and stalls the training kernels.  Flush on a CU-masked stream
        # (every `stride`-th CU) instead.
        stride = flush_cu_stride if flush_cu_stride is not None else int(
            os.environ.get("DWAMD_FLUSH_CU_STRIDE", "8"))
        # plain (default): a normal-priority torch stream.  lowprio: a
        # non-blocking lowest-priority stream -- with HIP's default 4 hardware
        # queues per process, once RCCL's communicator has taken queues, a
        # low-priority stream created afterwards ended up where the training
        # stream waits behind the flush (GPT2-1.5B steps after a save 109 ->
        # 150 ms; plain: 108, at 4 and 8 queues alike --
        # profiles/r5/flush_queue_sharing.md).  cumask: restrict the flush
        # blit to every `stride`-th CU (blocking stream type).
        kind = os.environ.get("DWAMD_FLUSH_STREAM", "plain")  # plain | lowprio | cumask | highprio
        self._cumask_ptr = None
        self.flush_cus = 0
        self.flush_stream_kind = kind
        if kind == "cumask" and stride > 1:
            n = ctypes.c_int(0)
            p = _kern().dw_stream_create_cumask(stride, ctypes.byref(n))
            if p:
                self._cumask_ptr = p
                self.flush_cus = n.value
        elif kind in ("lowprio", "highprio"):
            pr = ctypes.c_int(0)
            p = _kern().dw_stream_create_prio(0 if kind == "lowprio" else 2, ctypes.byref(pr))
            if p:
                self._cumask_ptr = p
        pre = _FLUSH_STREAMS.get(torch.device(device).index or 0) if kind == "plain" else None
        self.side_stream = (torch.cuda.ExternalStream(self._cumask_ptr, device=device) if self._cumask_ptr
                            else pre if pre is not None else torch.cuda.Stream(device=device))
        # "memcpy": hipMemcpyAsync (runtime blit); "kernel": our bounded
        # copy kernel storing through the device mapping of the pinned shm
        self.flush_mode = os.environ.get("DWAMD_FLUSH_MODE", "memcpy")
        self.flush_blocks = int(os.environ.get("DWAMD_FLUSH_BLOCKS", "64"))
        self.flush_stats: List[Tuple[int, float]] = []
        # (t_snapshot_enqueued, t_flush_start, t_flush_end, nbytes) per flush
        self.flush_log: List[tuple] = []
        self.pinned = PINNED
        # Future of the engine's background shm preparation (prefault +
        # hipHostRegister of this rank's slices): the flush -- never the
        # training pause -- waits for it.
        self.pending_prep: Optional[PrepTracker] = None
        # Snapshot staging in HBM.  Two buffers when the card has room (288 GB
        # MI355X: a 22 GB GPT2-1.5B state twice is nothing): snapshot k+1 then
        # never waits for the PCIe flush of snapshot k -- the flushes queue on
        # the single D2H thread and the training pause is just the HBM copy.
        # One buffer (the old wait-for-flush behaviour) when memory is tight.
        self._stagings: List[Optional[torch.Tensor]] = [None, None]
        self._ext = None  # HbmBuffer staging owned by a standby (hbm_tier.py)
        self._ext_key = None
        self._futures: List[Optional[Future]] = [None, None]
        self._flush_t0: List[float] = [0.0, 0.0]  # when each staging buffer's flush began moving bytes (0: not yet)
        self._flush_n: List[int] = [0, 0]
        self._nbuf = 0  # decided at the first snapshot
        self._next_stage = 0
        self.staging_reserve = int(os.environ.get("DWAMD_STAGING_RESERVE_GB", "24")) << 30
        self._executor = ThreadPoolExecutor(max_workers=1, thread_name_prefix="dwamd-d2h")
        self._desc_cache = {}
        # Overlapped snapshot (opt-in): the HBM->staging copy runs on its own
        # stream, concurrently with the next forward/backward (which only read
        # the checkpointed state), and the next optimizer step -- the first
        # writer -- waits for it through a global optimizer step pre-hook
        # (``fence``).  The training pause is then the host-side bookkeeping,
        # but the HBM-bound copy still takes its time from the next step
        # (GPT2-1.5B: pause 16 -> 9 ms, next step +7 ms): worth it only when
        # the step has HBM headroom to hide it.
        self.overlap = os.environ.get("DWAMD_OVERLAP_SNAPSHOT", "0") == "1"
        # grid of the overlapped ("late") copy: 0 = the whole chip (done
        # fastest, but it competes with the next forward); a few dozen blocks
        # trickle it through a few CUs during the ~100 ms before the fence
        self.overlap_blocks = int(os.environ.get("DWAMD_OVERLAP_BLOCKS", "0"))
        self._snap_stream: Optional[torch.cuda.Stream] = None
        self._fence_ev: Optional[torch.cuda.Event] = None
        # Bounded staging ring (``DWAMD_STAGING=ring``, or automatically when
        # not even one full-size staging buffer fits next to the model): K
        # chunks of C bytes of HBM instead of 1-2x the shard (_save_slice_ring)
        self.staging_mode = os.environ.get("DWAMD_STAGING", "auto")  # auto | full | ring
        self.ring_slots = max(2, int(os.environ.get("DWAMD_RING_SLOTS", "4")))
        self.ring_chunk = max(1 << 20, int(os.environ.get("DWAMD_RING_CHUNK_MB", "1024")) << 20)
        # HBM the ring may use in total: the part of the slice that fits in it
        # leaves the live tensors at HBM speed, only the rest drains at PCIe
        # speed before the next optimizer step (the fence).  0 = auto: in
        # ``auto`` staging the free HBM minus the reserve, in forced ``ring``
        # mode K x C
        self.ring_hbm = int(float(os.environ.get("DWAMD_RING_HBM_GB", "0")) * (1 << 30))
        self._ring_auto = 0
        self._ring: Optional[torch.Tensor] = None
        self._ring_free: List[torch.cuda.Event] = []
        self._ring_decision: Optional[Tuple[int, bool]] = None
        self._ring_gate: Optional[threading.Event] = None
        self._ring_last: dict = {}
        self._now_buf: Optional[torch.Tensor] = None
        self._ring_cache: dict = {}
        self.last_snapshot_mode = ""
        _install_fence_hook()

    @property
    def _staging(self) -> Optional[torch.Tensor]:
        return self._stagings[0]

    # ------------------------------------------------- HBM tier (hbm_tier.py)
    def _refresh_external(self, nbytes: int):
        """Snapshot into standby-owned buffers when available: this process's
        own (it was the standby) or the current standby's published ones.
        Switching waits for in-flight flushes of the old buffers."""
        from . import hbm_tier

        if nbytes <= 0:
            return
        cand, key = None, None
        own = [b for b in hbm_tier.OWNED if b.ptr and b.nbytes >= nbytes]
        # tier off: no standby-published buffers, but this process's own
        # (hbm_tier.reserve_private_staging while it was the standby) are its
        # staging -- no fresh VRAM on the first saves after a restart
        info = hbm_tier.find_published(os.environ.get("DWAMD_AGENT_CTL_DIR", ""),
                                       int(os.environ.get("LOCAL_RANK", "0"))) if (
            os.environ.get("DWAMD_HBM_TIER", "1") == "1") else None
        if info is not None and int(info["nbytes"]) >= nbytes and len(info["handles"]) >= 2:
            if info["_key"] == self._ext_key:
                return
            key = info["_key"]
        elif own and len(own) >= 2:
            if self._ext_key == ("own", os.getpid()):
                return
            cand, key = own[:2], ("own", os.getpid())
        else:
            return
        self.wait()
        if cand is None:
            cand = hbm_tier.import_published(info)
            if cand is None:
                self._ext_key = key  # do not retry a failing import every save
                return
        old = self._ext
        self._ext, self._ext_key = cand, key
        self._stagings = [cand[0], cand[1]]
        self._nbuf = 2
        self._next_stage = 0
        self._desc_cache.clear()
        for b in old or []:
            b.release()
        logger.info(f"checkpoint staging: using HBM buffers owned by pid {cand[0].owner_pid} "
                    f"({'own' if cand[0].owned else 'imported from the standby'})")

    def stage_owner(self, idx: int) -> int:
        b = self._stagings[idx] if idx < len(self._stagings) else None
        return getattr(b, "owner_pid", os.getpid())

    def _alloc(self, idx: int, nbytes: int) -> torch.Tensor:
        t = self._stagings[idx]
        if t is None or t.numel() < nbytes:
            self._stagings[idx] = None
            t = self._stagings[idx] = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        return t

    def staging(self, nbytes: int) -> torch.Tensor:
        """Buffer 0 (restore / gather path)."""
        self.wait()
        return self._alloc(0, nbytes)

    def _decide_buffers(self, nbytes: int):
        if self._nbuf:
            return
        nb = 1
        if os.environ.get("DWAMD_STAGING_BUFFERS", "auto") != "1":
            from .hbm_budget import staging_buffers

            try:
                free = device_free_bytes(self.device)
                have = sum(t.numel() for t in self._stagings if t is not None)
                nb = staging_buffers(free, have, nbytes, self.staging_reserve)
            except Exception:
                nb = 1
        self._nbuf = nb

    def wait(self):
        for i, f in enumerate(self._futures):
            if f is not None:
                f.result()
                self._futures[i] = None

    def wait_stage(self):
        """Wait only for the flush that last used the staging buffer the next
        snapshot will overwrite (all flushes with one buffer)."""
        if self._nbuf <= 1:
            return self.wait()
        f = self._futures[self._next_stage]
        if f is not None:
            f.result()
            self._futures[self._next_stage] = None

    def rewind_stage(self, idx: int):
        """The next snapshot reuses staging buffer ``idx`` (a discarded
        speculative snapshot already took it; no flush was queued for it)."""
        self._next_stage = idx % max(1, self._nbuf)

    def stage_busy_eta(self) -> float:
        """Seconds until the staging buffer the next snapshot uses is free:
        0 when idle; its flush's remaining bytes at the measured D2H rate when
        moving; +inf while that flush still waits (queue / shm preparation)."""
        if self._use_ring_cached():
            return 0.0
        idx = self._next_stage if self._nbuf > 1 else 0
        f = self._futures[idx] if idx < len(self._futures) else None
        if self._nbuf <= 1:
            pend = [i for i, x in enumerate(self._futures) if x is not None and not x.done()]
            if not pend:
                return 0.0
            idx = pend[-1]
            f = self._futures[idx]
        if f is None or f.done():
            return 0.0
        t0 = self._flush_t0[idx]
        if t0 <= 0.0:
            return float("inf")
        recent = self.flush_stats[-4:]
        rate = (sum(n for n, _ in recent) / max(1e-6, sum(t for _, t in recent))) if recent else 50e9
        return max(0.0, self._flush_n[idx] / rate - (time.perf_counter() - t0))

    def _use_ring_cached(self) -> bool:
        return self._ring_decision is not None and self._ring_decision[1]

    def busy(self) -> bool:
        return any(f is not None and not f.done() for f in self._futures)

    # ----------------------------------------------------------------- save
    def save_slice(self, layout: Layout, shm_payload_addr: int, lo: int, hi: int,
                   on_done: Callable[[], None], sync: bool = False,
                   before_copy: Optional[Callable[[int], None]] = None,
                   on_snapshot: Optional[Callable[[], None]] = None):
        """Snapshot payload bytes [lo, hi) of ``layout`` and flush to shm.
        ``before_copy(staging_idx)`` runs before the snapshot is enqueued
        (HBM-tier stamp invalidation); ``on_snapshot()`` on the flush thread
        once the snapshot sits complete in the staging buffer, before its
        PCIe flush (HBM-tier stamp: a standby-owned staging buffer survives
        this process, so the step is recoverable from then on)."""
        _flush_deferred_state()
        if self._use_ring(hi - lo):
            return self._save_slice_ring(layout, shm_payload_addr, lo, hi, on_done, sync)
        snap = self.snapshot(layout, lo, hi, before_copy)
        self.flush_snapshot(snap, shm_payload_addr, on_done, sync=sync, on_snapshot=on_snapshot)

    def snapshot(self, layout: Layout, lo: int, hi: int,
                 before_copy: Optional[Callable[[int], None]] = None) -> dict:
        """Enqueue the HBM->staging copy of payload bytes [lo, hi) (full
        staging mode) and return a handle for :meth:`flush_snapshot`.  The
        shm slot is not needed yet: the engine enqueues this first and picks /
        stamps the slot (gloo vote, metadata pickling) while the copy runs."""
        n = hi - lo
        _flush_deferred_state()  # a deferred-state optimizer writes its state back before a new snapshot
        self.last_snapshot_mode = "full"
        self._refresh_external(n)
        self._decide_buffers(n)
        self.wait_stage()  # this staging buffer's previous flush must have landed
        idx = self._next_stage
        self._next_stage = (idx + 1) % max(1, self._nbuf)
        self.last_stage = idx
        if before_copy is not None:
            before_copy(idx)
        cur = torch.cuda.current_stream(self.device)
        # a snapshot taken before the first optimizer step after a restart
        # must not read optimizer state a deferred restore is still landing
        from . import deferred_restore

        deferred_restore.wait_all(cur, self.device)
        copy_stream = cur
        if self.overlap and n > 0:
            if self._snap_stream is None:
                self._snap_stream = _snapshot_stream(self.device)
            copy_stream = self._snap_stream
            copy_stream.wait_stream(cur)  # the state as of this save call
            for e in _pending_updates(self.device):  # ... after an overlapped update
                copy_stream.wait_event(e)
        else:
            from ..optimizers.overlap import join_all

            join_all(cur)
        stg = None
        if n > 0:
            stg = self._alloc(idx, n)
            base = stg.data_ptr()
            overlapped = copy_stream is not cur
            key = (layout.signature, lo, hi, base, tuple(e.src_ptr for e in layout.extents), overlapped,
                   len(_OPTIMIZERS) if overlapped else 0)
            descs = self._desc_cache.get(key)
            if descs is None:
                pieces = [(e.src_ptr + (a - e.offset), base + (a - lo), b - a)
                          for e, a, b in intersect_extents(layout.gpu_extents(), lo, hi)]
                if overlapped:
                    # only storages that just an optimizer step writes may be
                    # read after this call returns; the rest is copied now
                    rng = _step_only_ranges()
                    starts = [a for a, _b in rng]
                    late = [p for p in pieces if _covered(rng, starts, p[0], p[2])]
                    now = [p for p in pieces if not _covered(rng, starts, p[0], p[2])]
                    descs = (build_descs(now, self.device), build_descs(late, self.device))
                else:
                    descs = (build_descs(pieces, self.device), None)
                if len(self._desc_cache) >= 4:  # one entry per staging buffer (+ slack)
                    self._desc_cache.pop(next(iter(self._desc_cache)))
                self._desc_cache[key] = descs
            launch_multi_copy(descs[0], cur)
            if descs[1] is not None:
                copy_stream.wait_stream(cur)  # the "now" part is ordered before the flush too
                launch_multi_copy(descs[1], copy_stream, self.overlap_blocks)
        ev = torch.cuda.Event()
        ev.record(copy_stream)
        if copy_stream is not cur:
            self._fence_ev = ev
            _FENCED.add(self)
        return {"layout": layout, "lo": lo, "hi": hi, "idx": idx, "stg": stg, "ev": ev,
                "t_enq": time.perf_counter()}

    def flush_snapshot(self, snap: dict, shm_payload_addr: int, on_done: Callable[[], None], sync: bool = False,
                       on_snapshot: Optional[Callable[[], None]] = None):
        """Copy the CPU extents into the shm slot now and queue the PCIe flush
        of the staged bytes behind the snapshot's event."""
        layout, lo, hi, idx, stg, ev = (snap[k] for k in ("layout", "lo", "hi", "idx", "stg", "ev"))
        n = hi - lo
        # the PCIe flush writes the device region only: host tensors (below)
        # sit after it in the payload and must not be overwritten with the
        # staging buffer's bytes at their offsets
        n_dev = max(0, min(hi, layout.gpu_end) - lo)
        t_enq = snap["t_enq"]
        if n > 0:
            # CPU tensors go straight to shm (small: counters, rng state...)
            for e, a, b in intersect_extents(layout.cpu_extents(), lo, hi):
                runtime().dw_memcpy_parallel(ctypes.c_void_p(shm_payload_addr + a),
                                             ctypes.c_void_p(e.src_ptr + (a - e.offset)), b - a, 4)
        prep = self.pending_prep

        # NOTE: every host-side wait in this thread goes through ctypes (which
        # drops the GIL); torch's Stream/Event.synchronize would hold the GIL
        # for the whole PCIe transfer and stall the training thread's launches.
        def flush():
            t_start = time.perf_counter()
            if n > 0:
                if on_snapshot is not None:
                    _check(_kern().dw_event_sync(ctypes.c_void_p(ev.cuda_event)), "snapshot sync")
                    on_snapshot()
                    delay = float(os.environ.get("DWAMD_FAULT_FLUSH_DELAY_S", "0") or 0)
                    if delay > 0:
                        # fault injection: a slow PCIe flush, so a kill lands
                        # after the snapshot and before the shm copy completes
                        time.sleep(delay)
                if prep is not None:
                    prep.wait(shm_payload_addr + lo, n)  # this range's prefault + registration
                # registering here (flush thread), not in the training pause:
                # a no-op once the range is covered
                pinned = self.pinned.ensure(shm_payload_addr + lo, n)
                with torch.cuda.stream(self.side_stream):
                    self.side_stream.wait_event(ev)  # device-side dependency only
                    t0 = time.perf_counter()
                    self._flush_t0[idx], self._flush_n[idx] = t0, n_dev
                    dst = shm_payload_addr + lo
                    src = stg.data_ptr()
                    sp = ctypes.c_void_p(self.side_stream.cuda_stream)
                    segs = (self.pinned.split(dst, n_dev) if pinned else [(dst, n_dev, False)]) if n_dev else []
                    dptr = _kern().dw_host_device_ptr(ctypes.c_void_p(dst)) if (
                        pinned and self.flush_mode == "kernel" and len(segs) == 1) else None
                    if dptr and (n_dev % 16 == 0):
                        _check(_kern().dw_stream_copy(ctypes.c_void_p(dptr), ctypes.c_void_p(src), n_dev,
                                                      self.flush_blocks, sp), "D2H flush")
                    else:
                        for a, c, p in segs:
                            _check(_kern().dw_memcpy_async(ctypes.c_void_p(a), ctypes.c_void_p(src + (a - dst)), c,
                                                           1 if p else 3, sp), "D2H flush")
                _check(_kern().dw_stream_sync(ctypes.c_void_p(self.side_stream.cuda_stream)), "flush sync")
                t1 = time.perf_counter()
                self.flush_stats.append((n_dev, t1 - t0))
                # (+ when the flush thread took it up, pinned bytes of the destination)
                self.flush_log.append((t_enq, t0, t1, n_dev, t_start, sum(c for _a, c, p in segs if p)))
            else:
                with torch.cuda.stream(self.side_stream):
                    self.side_stream.wait_event(ev)
                _check(_kern().dw_stream_sync(ctypes.c_void_p(self.side_stream.cuda_stream)), "flush sync")
            on_done()

        self._flush_t0[idx] = 0.0
        if sync:
            self.wait()
            flush()
        else:
            self._futures[idx] = self._executor.submit(flush)

    def fence(self):
        """Make the current stream wait for a pending overlapped snapshot
        (called before anything may write the checkpointed state)."""
        gate = self._ring_gate
        if gate is not None:
            # the ring's last chunk copy is enqueued by the flush thread
            gate.wait()
            self._ring_gate = None
            ev = self._ring_last.pop("ev", None)
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
        ev = self._fence_ev
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            self._fence_ev = None

    # ------------------------------- ring progress (deferred-state optimizers)
    def ring_pending(self) -> bool:
        """A ring snapshot whose chunk copies may not all have run yet."""
        return self._ring_gate is not None

    def _ring_wait_enqueued(self):
        gate = self._ring_gate
        if gate is not None:
            gate.wait()  # the flush thread has enqueued every chunk copy (host side, quick)

    def ring_done(self) -> bool:
        """Every chunk of the pending ring snapshot has been copied (its
        sources may be written again)."""
        if self._ring_gate is None:
            return True
        self._ring_wait_enqueued()
        ev = self._ring_last.get("ev")
        return ev is None or ev.query()

    def ring_sources(self) -> List[Tuple[int, int]]:
        """Device address ranges the pending ring snapshot reads."""
        chunks = getattr(self, "_ring_chunks", None)
        if chunks is None or self._ring_gate is None:
            return []
        return _merge([r for srcs in chunks[0] for r in srcs])

    def ring_staged(self) -> List[Tuple[int, int]]:
        """Source ranges already copied into the ring (chunk events done at
        the time of the call: a lower bound)."""
        chunks = getattr(self, "_ring_chunks", None)
        if chunks is None or self._ring_gate is None:
            return []
        self._ring_wait_enqueued()
        srcs, evs = chunks
        return _merge([r for j, ev in enumerate(evs) if ev is not None and ev.query() for r in srcs[j]])

    def ring_wait_ranges(self, ranges: List[Tuple[int, int]], stream=None):
        """Order ``stream`` (default: current) after the chunk copies that
        read any of ``ranges`` (device-side waits)."""
        chunks = getattr(self, "_ring_chunks", None)
        if chunks is None or self._ring_gate is None:
            return
        self._ring_wait_enqueued()
        stream = stream or torch.cuda.current_stream(self.device)
        srcs, evs = chunks
        for j, ev in enumerate(evs):
            if ev is not None and any(a < hi and lo < b for a, b in srcs[j] for lo, hi in ranges):
                stream.wait_event(ev)

    def ring_last_event(self):
        self._ring_wait_enqueued()
        return self._ring_last.get("ev")

    # ------------------------------------------------------- staging ring
    def _use_ring(self, n: int) -> bool:
        if n <= 0 or self.staging_mode == "full":
            return False
        if self.staging_mode == "ring":
            return True
        if self._ring_decision is not None and self._ring_decision[0] == n:
            return self._ring_decision[1]
        ring = False
        # standby-owned staging (this process's own after an activation, or
        # the current standby's) needs no HBM of this process: adopt it before
        # judging free memory -- right after a restart the dead worker's HBM
        # may not be released yet, and a ring decided then (cached per slice
        # size) would fence every later optimizer step on its PCIe drain
        self._refresh_external(n)
        if self._ext is None:
            try:
                free = device_free_bytes(self.device)
                have = sum(t.numel() for t in self._stagings if t is not None)
                from .hbm_budget import use_ring

                ring = use_ring(free, have, n, self.staging_reserve)
                self._ring_auto = max(0, free + have - self.staging_reserve)
            except Exception:
                ring = False
        self._ring_decision = (n, ring)
        if ring:
            self.wait()
            self._stagings = [None, None]  # give full-size buffers back
            K, C = self._ring_shape(n)
            logger.info(f"checkpoint staging: {n / 2**30:.1f} GiB slice does not fit in HBM next to the model; "
                        f"bounded ring of {K} x {C >> 20} MiB")
        return ring

    def _ring_shape(self, n: int) -> Tuple[int, int]:
        """(slots K, chunk bytes C) of the ring for an n-byte slice: at least
        DWAMD_RING_SLOTS x DWAMD_RING_CHUNK_MB, grown to the HBM budget (never
        beyond the slice)."""
        K, C = self.ring_slots, self.ring_chunk
        C = min(C, max(16, (n + K - 1) // K + 15 & ~15))  # tiny slices: no oversized ring
        budget = self.ring_hbm or (self._ring_auto if self.staging_mode == "auto" else 0)
        if budget > K * C:
            K = max(K, min(budget, n) // C)
        return K, C

    @property
    def staging_hbm_bytes(self) -> int:
        """HBM this copier holds for snapshot staging right now."""
        b = sum(t.numel() for t in self._stagings if t is not None)
        if self._ring is not None:
            b += self._ring.numel()
        if self._now_buf is not None:
            b += self._now_buf.numel()
        return b

    def _save_slice_ring(self, layout: Layout, shm_payload_addr: int, lo: int, hi: int,
                         on_done: Callable[[], None], sync: bool):
        """Snapshot through K x C bytes of HBM.

        The slice streams chunk by chunk: a copy stream gathers chunk j from
        the live tensors into ring slot j % K (after slot j % K's previous
        D2H has drained, a device-side event wait) and the flush stream DMAs
        it to pinned shm.  Nothing is copied before this call returns except
        storages that something other than ``Optimizer.step`` may write
        (buffers): those go into a small HBM side buffer on the compute
        stream first.  Parameters and optimizer state are read by the ring
        while forward/backward run; the next optimizer step is fenced on the
        last chunk copy (global step pre-hook).  If the non-optimizer part
        exceeds one chunk (e.g. no optimizer has stepped yet), the call
        blocks until the ring has drained.  Host-side enqueueing happens on
        the flush thread (it also waits for the shm registration), so the
        training thread never waits on PCIe unless it reaches the fence."""
        self.last_snapshot_mode = "ring"
        hi_all = hi
        hi = max(lo, min(hi, layout.gpu_end))  # the ring carries the device region; host tensors go to shm below
        n = hi - lo
        self.wait()  # one ring: the previous pipeline must have drained
        self.fence()
        K, C = self._ring_shape(n)
        if self._ring is None or self._ring.numel() < K * C:
            self._ring = None
            self._ring = torch.empty(K * C, dtype=torch.uint8, device=self.device)
            self._ring_free = [torch.cuda.Event() for _ in range(K)]
            self._ring_cache.clear()
        if self._snap_stream is None:
            self._snap_stream = _snapshot_stream(self.device)
        cur = torch.cuda.current_stream(self.device)
        cstream = self._snap_stream
        ring_base = self._ring.data_ptr()

        gpu = [(e.src_ptr + (a - e.offset), a - lo, b - a) for e, a, b in intersect_extents(layout.gpu_extents(), lo, hi)]
        rng = _step_only_ranges()
        starts = [a for a, _b in rng]
        now = [p for p in gpu if not _covered(rng, starts, p[0], p[2])]
        now_bytes = sum(p[2] for p in now)
        blocking = sync or now_bytes > C
        if not blocking and now:
            if self._now_buf is None or self._now_buf.numel() < now_bytes:
                self._now_buf = torch.empty(max(now_bytes, 1 << 20), dtype=torch.uint8, device=self.device)
        nb = self._now_buf.data_ptr() if (self._now_buf is not None and not blocking and now) else 0
        key = (layout.signature, lo, hi, tuple(e.src_ptr for e in layout.extents), ring_base, C, nb, blocking,
               len(_OPTIMIZERS or ()))
        plan = self._ring_cache.get(key)
        if plan is None:
            now_set = set(now)
            srcs, now_descs, k = [], [], 0
            for p in gpu:
                if nb and p in now_set:
                    now_descs.append((p[0], nb + k, p[2]))
                    srcs.append((nb + k, p[1], p[2]))
                    k += p[2]
                else:
                    srcs.append(p)
            srcs.sort(key=lambda x: x[1])
            rows, bounds = [], []
            nchunks = (n + C - 1) // C
            i = 0
            for j in range(nchunks):
                c0, c1 = j * C, min(n, (j + 1) * C)
                r0 = len(rows)
                while i < len(srcs) and srcs[i][1] + srcs[i][2] <= c0:
                    i += 1
                t = i
                while t < len(srcs) and srcs[t][1] < c1:
                    s_, off, ln = srcs[t]
                    a_, b_ = max(off, c0), min(off + ln, c1)
                    o = a_
                    while o < b_:  # CHUNK-sized descriptor rows
                        c = min(CHUNK, b_ - o)
                        rows.append((s_ + (o - off), ring_base + (j % K) * C + (o - c0), c))
                        o += c
                    t += 1
                bounds.append((r0, len(rows), c0, c1))
            # per chunk: the merged source address ranges it copies (what a
            # deferred-state optimizer asks about, see ring_staged)
            chunk_src = [_merge([(r[0], r[0] + r[2]) for r in rows[b0:b1]]) for b0, b1, _c0, _c1 in bounds]
            descs = (torch.from_numpy(np.asarray(rows, dtype=np.uint64).view(np.int64)).to(self.device)
                     if rows else torch.empty(0, 3, dtype=torch.int64, device=self.device))
            plan = (descs, bounds, build_descs(now_descs, self.device) if now_descs else None, chunk_src)
            if len(self._ring_cache) >= 4:
                self._ring_cache.pop(next(iter(self._ring_cache)))
            self._ring_cache[key] = plan
        descs, bounds, now_d, chunk_src = plan
        chunk_evs: List[Optional[torch.cuda.Event]] = [None] * len(bounds)
        self._ring_chunks = (chunk_src, chunk_evs)
        if now_d is not None:
            launch_multi_copy(now_d, cur)  # forward-written storages: copied before returning
        for e, a, b in intersect_extents(layout.cpu_extents(), lo, hi_all):
            runtime().dw_memcpy_parallel(ctypes.c_void_p(shm_payload_addr + a),
                                         ctypes.c_void_p(e.src_ptr + (a - e.offset)), b - a, 4)
        ev_start = torch.cuda.Event()
        ev_start.record(cur)
        # parameters / optimizer state after an overlapped update; waited on
        # by the flush thread before the gate opens (the next step, which
        # re-records these events, is fenced on the gate)
        pend = _pending_updates(self.device)
        prep = self.pending_prep
        gate = threading.Event()
        holder = self._ring_last
        holder.pop("ev", None)
        free = self._ring_free
        t_enq = time.perf_counter()

        def flush():
            try:
                if prep is not None:
                    prep.wait(shm_payload_addr + lo, n)
                pinned = self.pinned.ensure(shm_payload_addr + lo, n)
                sp = ctypes.c_void_p(self.side_stream.cuda_stream)
                t0 = time.perf_counter()
                cstream.wait_event(ev_start)
                for e in pend:
                    cstream.wait_event(e)
                for j, (r0, r1, c0, c1) in enumerate(bounds):
                    if j >= K:
                        cstream.wait_event(free[j % K])  # slot's previous D2H has landed
                    launch_multi_copy(descs[r0:r1], cstream)
                    ready = torch.cuda.Event()
                    ready.record(cstream)
                    chunk_evs[j] = ready
                    self.side_stream.wait_event(ready)
                    dst = shm_payload_addr + lo + c0
                    src = ring_base + (j % K) * C
                    for a_, c_, p_ in (self.pinned.split(dst, c1 - c0) if pinned else [(dst, c1 - c0, False)]):
                        _check(_kern().dw_memcpy_async(ctypes.c_void_p(a_), ctypes.c_void_p(src + (a_ - dst)), c_,
                                                       1 if p_ else 3, sp), "ring D2H")
                    free[j % K].record(self.side_stream)
                last = torch.cuda.Event()
                last.record(cstream)
                holder["ev"] = last
            finally:
                gate.set()
            _check(_kern().dw_stream_sync(ctypes.c_void_p(self.side_stream.cuda_stream)), "ring flush sync")
            t1 = time.perf_counter()
            self.flush_stats.append((n, t1 - t0))
            self.flush_log.append((t_enq, t0, t1, n))
            on_done()

        self._ring_gate = gate
        _FENCED.add(self)
        self._futures[0] = self._executor.submit(flush)
        if blocking:
            self._futures[0].result()
            self._futures[0] = None
            self.fence()

    # ----------------------------------------------------------------- load
    def restore(self, pieces_gpu: List[Tuple[int, int, int]], shm_payload_addr: int, payload_bytes: int,
                lo: int, hi: int, gather_group=None, world: int = 1, hbm_src: Optional[int] = None):
        """Restore GPU targets.

        pieces_gpu: (payload_off, dst_addr, nbytes) for every GPU target.
        If ``gather_group`` is None this process copies every piece itself
        (H2D straight into the targets).  Otherwise this process H2D's only
        its slice [lo, hi) into a full-size temporary buffer, the group
        all-gathers, and one kernel scatters into the targets.
        ``hbm_src``: device address of an HBM-tier buffer holding payload
        bytes [lo, hi) of the step being restored -- the slice is then copied
        device-to-device (multi-copy kernel) instead of H2D from shm.
        """
        self.fence()  # the restore overwrites the state a pending snapshot still reads
        cur = torch.cuda.current_stream(self.device)
        from ..optimizers.overlap import join_all

        join_all(cur)  # ... and a pending overlapped optimizer update would overwrite it
        from . import deferred_restore

        deferred_restore.wait_all(cur, self.device)  # ... as would a previous restore's late copies
        if gather_group is None or world <= 1:
            merged = _merge_pieces(pieces_gpu)
            if hbm_src is not None:
                launch_multi_copy(build_descs([(hbm_src + (off - lo), dst, n) for off, dst, n in merged],
                                              self.device), cur)
            else:
                self._pipelined_h2d([(shm_payload_addr + off, dst, n) for off, dst, n in merged], cur)
            return
        import torch.distributed as dist

        from .gather import all_gather_slices
        from .hbm_budget import gather_chunk

        from . import hbm_tier

        per = hi - lo
        rank = dist.get_rank(gather_group)
        # the gather's temporary (never the staging buffers: with the HBM tier
        # they hold the checkpoint being restored) is bounded: world x c bytes
        # per round (hbm_budget.gather_chunk), the whole payload in one round
        # when it fits.  c is a COLLECTIVE size: it depends on (per, world,
        # DWAMD_RESTORE_GATHER_GB) only, never on this rank's free memory, so
        # every rank runs the same rounds.  A standby reserved the temporary
        # while parked (hbm_tier.reserve_restore_temp): no fresh VRAM on the
        # restart path
        c = min(per, gather_chunk(per, world, 1 << 62))
        tmp = hbm_tier.take_restore_temp()
        want_idx = torch.device(self.device).index
        if (tmp is not None and tmp.is_cuda and (want_idx is None or tmp.device.index == want_idx)
                and tmp.numel() >= c * world):
            self.last_restore_temp = "reserved"
        else:
            tmp = torch.empty(c * world, dtype=torch.uint8, device=self.device)
            self.last_restore_temp = "allocated"
        merged = _merge_pieces(pieces_gpu)
        self.last_restore_gather = {"rounds": -(-per // c) if per else 0, "chunk": c, "temp_bytes": c * world}
        for o in range(0, per, c):
            n = min(c, per - o)
            buf = tmp[: n * world]
            # every rank's slice has the same size ``per`` (the last one may be
            # short in payload terms, padded): copy what exists of this round
            real = max(0, min(lo + o + n, payload_bytes) - (lo + o))
            dst0 = buf.data_ptr() + rank * n
            if real > 0:
                if hbm_src is not None:
                    launch_multi_copy(build_descs([(hbm_src + o, dst0, real)], self.device), cur)
                else:
                    self._pipelined_h2d([(shm_payload_addr + lo + o, dst0, real)], cur)
            self.last_restore_gather["transport"] = all_gather_slices(buf, buf[rank * n: (rank + 1) * n],
                                                                      gather_group)
            base = buf.data_ptr()
            scatter = []
            for r in range(world):
                a, b = r * per + o, r * per + o + n  # payload bytes of rank r's part of this round
                for off, dst, m in merged:
                    x0, x1 = max(a, off), min(b, off + m)
                    if x0 < x1:
                        scatter.append((base + r * n + (x0 - a), dst + (x0 - off), x1 - x0))
            launch_multi_copy(build_descs(scatter, self.device), cur)
        del tmp

    def restore_deferred(self, pieces_gpu: List[Tuple[int, int, int]], shm_payload_addr: int, t0: float):
        """H2D of ``pieces_gpu`` (payload_off, dst_addr, nbytes) from the shm
        slot on a side stream, ordered after everything queued on the current
        stream so far (the restore() of the other pieces included).  Returns
        the registered ``deferred_restore.DeferredRestore``."""
        from . import deferred_restore

        cur = torch.cuda.current_stream(self.device)
        # on the flush stream (idle at a restore; the first flush queues
        # behind these copies): a stream created here, after RCCL's, shared a
        # hardware queue with an import standby's compute stream at HIP's
        # default 4 queues, and every step after a save then waited for that
        # save's 0.4 s flush (import-mode goodput 73 -> 47 %,
        # profiles/r6/import_stall_ab.jsonl)
        merged = _merge_pieces(pieces_gpu)
        copies = [(shm_payload_addr + off, dst, n) for off, dst, n in merged]
        d = deferred_restore.DeferredRestore(self.device, self.side_stream, cur.record_event(),
                                             lambda stream: self._pipelined_h2d(copies, stream), t0)
        deferred_restore.add(d)
        return d

    def write_back(self, dev_src: int, host_dst: int, nbytes: int):
        """D2H of ``nbytes`` from a device address into (shm) host memory,
        synchronous (pinned in chunks like the flush)."""
        if nbytes <= 0:
            return
        cur = torch.cuda.current_stream(self.device)
        sp = ctypes.c_void_p(cur.cuda_stream)
        pinned = self.pinned.ensure(host_dst, nbytes)
        for a, c, p in (self.pinned.split(host_dst, nbytes) if pinned else [(host_dst, nbytes, False)]):
            _check(_kern().dw_memcpy_async(ctypes.c_void_p(a), ctypes.c_void_p(dev_src + (a - host_dst)), c,
                                           1 if p else 3, sp), "D2H write-back")
        _check(_kern().dw_stream_sync(sp), "D2H write-back sync")

    def _pipelined_h2d(self, copies: List[Tuple[int, int, int]], stream, chunk: int = 512 << 20):
        """H2D of (host_src, dev_dst, nbytes) ranges.  Pinning (hipHostRegister,
        ~50 GB/s) of chunk k+1 overlaps the DMA (~57 GB/s) of chunk k, so a
        freshly restarted process pays ~max(pin, copy) instead of the sum."""
        pieces = []
        for src, dst, n in copies:
            o = 0
            while o < n:
                c = min(chunk, n - o)
                pieces.append((src + o, dst + o, c))
                o += c
        if not pieces:
            return
        with ThreadPoolExecutor(max_workers=1, thread_name_prefix="dwamd-pin") as ex:
            futs = [ex.submit(self.pinned.ensure, s, n) for s, _d, n in pieces]
            sp = ctypes.c_void_p(stream.cuda_stream)
            for (s, d, n), f in zip(pieces, futs):
                pinned = f.result()
                for a, c, p in (self.pinned.split(s, n) if pinned else [(s, n, False)]):
                    _check(_kern().dw_memcpy_async(ctypes.c_void_p(d + (a - s)), ctypes.c_void_p(a), c,
                                                   0 if p else 3, sp), "H2D restore")

    def close(self):
        try:
            # an optimizer still deferring state behind this copier's ring
            # writes it back now; then nothing pending may outlive the copier
            # (a closed copier left in the fence set would be offered to
            # later optimizers)
            try:
                _flush_deferred_state()
            except Exception as e:  # e.g. at interpreter exit, the runtime already torn down
                logger.warning(f"deferred optimizer-state write-back at close failed: {e}")
            self.wait()
            self.fence()
        finally:
            if _FENCED is not None:
                _FENCED.discard(self)
            self._executor.shutdown(wait=True)
            self.pinned.release_all()
            self._stagings = [None, None]
            self._ring = None
            self._now_buf = None
            for b in self._ext or []:
                b.release()
            self._ext = None
            if self._cumask_ptr:
                self.side_stream.synchronize()
                _kern().dw_stream_destroy(ctypes.c_void_p(self._cumask_ptr))
                self._cumask_ptr = None


def _merge_pieces(pieces: List[Tuple[int, int, int]]) -> List[Tuple[int, int, int]]:
    ps = sorted(pieces)
    out: List[List[int]] = []
    for off, dst, n in ps:
        if out and out[-1][0] + out[-1][2] == off and out[-1][1] + out[-1][2] == dst:
            out[-1][2] += n
        else:
            out.append([off, dst, n])
    return [tuple(x) for x in out]


def match_targets(meta_tree, target) -> Tuple[List[Tuple[TensorMeta, torch.Tensor]], bool]:
    """Pair TensorMeta leaves with same-shaped tensors of ``target`` (same
    tree structure).  Returns (pairs, structure_ok)."""
    metas = iter_leaves(meta_tree)
    tgts = iter_leaves(target)
    if len(metas) != len(tgts):
        return [], False
    pairs = []
    for m, t in zip(metas, tgts):
        if isinstance(m, TensorMeta):
            if not torch.is_tensor(t) or t.numel() != m.numel or t.dtype != m.dtype:
                return [], False
            pairs.append((m, t))
    return pairs, True
