"""HBM checkpoint tier: snapshot staging buffers that outlive the worker.

Every flash save first copies this rank's payload slice HBM -> HBM into a
staging buffer (``copier.py``), then flushes it to pinned host shm over PCIe.
On MI355X (288 GB HBM per GPU) those staging buffers can live in memory that
is *not* owned by the training process: the local rank's deep warm standby
(``elastic_agent/standby.py``) allocates them with ``hipMalloc`` and
publishes dmabuf IPC handles; the live worker imports them and snapshots
into them.  When the worker dies, the buffers -- holding the latest complete
checkpoint -- stay alive in the standby, which becomes the next worker and
restores with a device-to-device copy (~10 ms for a 22 GB GPT2-1.5B state at
~4 TB/s) instead of a PCIe H2D from shm (~0.4 s at ~55 GB/s).  The host shm
copy is still written for durability against losing the GPU or the node.

Validity is tracked per (slice, staging buffer) with stamp words in the
checkpoint segment's header (``HBM_STAMP_BASE``): (step, owner pid, bytes).
A buffer's stamp is zeroed before a snapshot is written into it and set
only after the flush of that snapshot completed, i.e. exactly when the
matching shm slot becomes complete.  A restoring process uses a buffer only
if it owns it (pid match) and the stamp names the step every rank agreed to
restore; otherwise it falls back to the shm H2D path.

There is no reference counterpart (the reference keeps one host-memory copy,
``ckpt_saver.py:SharedMemoryHandler``); this is an MI355X-first tier.
"""

import ctypes
import json
import os
from typing import List, Optional

from ..common.log import logger

PUBLISH_PREFIX = "hbm_staging."
HBM_STAMP_BASE = 4096  # header word index (int64) of slice 0 / buffer 0
STAMP_WORDS = 4  # step, owner pid, nbytes, reserved
MAX_STAMP_SLICES = 256


def _kern():
    from .._native import kernels

    return kernels(required=True)


def stamp_index(slice_idx: int, buf: int) -> int:
    return HBM_STAMP_BASE + (slice_idx * 2 + buf) * STAMP_WORDS


class HbmBuffer:
    """A raw device allocation usable as a copier staging buffer."""

    def __init__(self, ptr: int, nbytes: int, owner_pid: int, owned: bool):
        self.ptr = ptr
        self.nbytes = nbytes
        self.owner_pid = owner_pid
        self.owned = owned  # hipMalloc'ed by this process (else IPC-imported)

    def data_ptr(self) -> int:
        return self.ptr

    def numel(self) -> int:
        return self.nbytes

    def release(self):
        if not self.ptr:
            return
        if self.owned:
            _kern().dw_device_free(ctypes.c_void_p(self.ptr))
        else:
            _kern().dw_ipc_close_handle(ctypes.c_void_p(self.ptr))
        self.ptr = 0


# buffers this process allocated while it was a standby (adopted as staging
# by its own copier after activation)
OWNED: List[HbmBuffer] = []
_published_key = None


def _free_hbm() -> int:
    f, t = ctypes.c_uint64(0), ctypes.c_uint64(0)
    if _kern().dw_mem_get_info(ctypes.byref(f), ctypes.byref(t)) != 0:
        return 0
    return int(f.value)


_warmed = False


def _warm_restore_path():
    """One tiny multi-copy in the standby: loads the copy kernel's code
    object and the descriptor upload path now, not inside the restore that
    follows the standby's activation."""
    global _warmed
    if _warmed:
        return
    try:
        import torch

        from .copier import build_descs, launch_multi_copy

        t = torch.zeros(2, 4096, dtype=torch.uint8, device="cuda")
        launch_multi_copy(build_descs([(t[0].data_ptr(), t[1].data_ptr(), 4096)], t.device))
        torch.cuda.synchronize()
        _warmed = True
    except Exception as e:  # never fatal
        logger.warning(f"standby: restore-path warm-up failed: {e}")


def _alloc_owned(nbytes: int, nbuf: int) -> bool:
    for _ in range(nbuf):
        p = ctypes.c_void_p(0)
        err = _kern().dw_device_malloc(nbytes, ctypes.byref(p))
        if err != 0:
            logger.warning(f"standby: hipMalloc({nbytes}) failed ({err})")
            release_owned()
            return False
        OWNED.append(HbmBuffer(int(p.value), nbytes, os.getpid(), owned=True))
    return True


def release_owned():
    global _published_key
    for b in OWNED:
        b.release()
    OWNED.clear()
    _published_key = None


def publish_standby_buffers(ctl_dir: str, local_rank: int, nbytes: int, nbuf: int = 2,
                            reserve: int = 24 << 30) -> bool:
    """Standby side: (re)allocate ``nbuf`` buffers of ``nbytes`` and publish
    their IPC handles in ``ctl_dir``.  No-op if already published at that
    size; False if HBM is too tight (the worker keeps its own buffers)."""
    global _published_key
    if not ctl_dir or nbytes <= 0:
        return False
    key = (nbytes, nbuf, True)
    if _published_key == key and OWNED:
        return True
    release_owned()
    if _free_hbm() < nbuf * nbytes + reserve:
        logger.info(f"standby: not enough free HBM for {nbuf} x {nbytes} B checkpoint staging")
        return False
    hsz = _kern().dw_ipc_handle_size()
    if not _alloc_owned(nbytes, nbuf):
        return False
    handles = []
    for buf in OWNED:
        h = ctypes.create_string_buffer(hsz)
        err = _kern().dw_ipc_get_handle(ctypes.c_void_p(buf.ptr), h)
        if err != 0:
            logger.warning(f"standby: hipIpcGetMemHandle failed ({err}); HBM tier disabled")
            release_owned()
            return False
        handles.append(h.raw.hex())
    info = {"pid": os.getpid(), "nbytes": nbytes, "handles": handles}
    path = os.path.join(ctl_dir, f"{PUBLISH_PREFIX}{local_rank}.json")
    with open(path + ".tmp", "w") as f:
        json.dump(info, f)
    os.replace(path + ".tmp", path)
    _published_key = key
    _warm_restore_path()
    logger.info(f"standby: published {nbuf} x {nbytes / 2**30:.1f} GiB HBM checkpoint staging buffers")
    return True


def reserve_private_staging(nbytes: int, nbuf: int = 2, reserve: int = 24 << 30) -> bool:
    """HBM tier off (``DWAMD_HBM_TIER=0``, the reference's restart
    semantics): the standby still allocates the staging buffers that the
    worker it becomes will snapshot into -- privately (no handles
    published; the live worker keeps its own).  The first saves after a
    restart then need no fresh VRAM: a hipMalloc of a 20 GB buffer next to a
    killed process whose VRAM the driver is still tearing down stalled
    0.5-3 s (BENCH_r05 ``import_mode.save_ms_after_restart`` 515, 491 ms).
    The copier adopts them as its own staging (``copier._refresh_external``)."""
    global _published_key
    if nbytes <= 0:
        return False
    key = (nbytes, nbuf, False)
    if _published_key == key and OWNED:
        return True
    release_owned()
    if _free_hbm() < nbuf * nbytes + reserve:
        logger.info(f"standby: not enough free HBM for {nbuf} x {nbytes} B private checkpoint staging")
        return False
    if not _alloc_owned(nbytes, nbuf):
        return False
    _published_key = key
    _warm_restore_path()
    logger.info(f"standby: reserved {nbuf} x {nbytes / 2**30:.1f} GiB HBM checkpoint staging (private)")
    return True


# ------------------------------------------------ restore-time reservations
# The replicated restore's all-gather temporary (copier.restore, N > 1):
# allocated by the standby while parked, handed to the restore, then freed
# into the caching allocator (where the first step's activations reuse it).
_RESTORE_TMP = None


def reserve_restore_temp(nbytes: int, reserve: int = 24 << 30) -> int:
    """Hold ``nbytes`` of HBM for the restore's gather temporary (bytes held)."""
    global _RESTORE_TMP
    if nbytes <= 0:
        return 0
    if _RESTORE_TMP is not None and _RESTORE_TMP.numel() >= nbytes:
        return _RESTORE_TMP.numel()
    import torch

    _RESTORE_TMP = None
    if _free_hbm() < nbytes + reserve:
        return 0
    _RESTORE_TMP = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    return nbytes


def take_restore_temp():
    """The reserved gather temporary (once), or None."""
    global _RESTORE_TMP
    t, _RESTORE_TMP = _RESTORE_TMP, None
    return t


def reserve_small_pool(mib: int = 128):
    """Pre-fill the caching allocator's small-block pool (2 MiB segments for
    allocations <= 1 MiB: descriptor tables, scalars, the first batch) so
    the restart path allocates none of them from the driver."""
    import torch

    ts = [torch.empty(1 << 20, dtype=torch.uint8, device="cuda") for _ in range(max(1, mib))]
    del ts


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def find_published(ctl_dir: str, local_rank: int) -> Optional[dict]:
    if not ctl_dir:
        return None
    path = os.path.join(ctl_dir, f"{PUBLISH_PREFIX}{local_rank}.json")
    try:
        st = os.stat(path)
        with open(path) as f:
            info = json.load(f)
    except (OSError, ValueError):
        return None
    info["_key"] = (info.get("pid"), st.st_mtime_ns, tuple(info.get("handles", ())))
    if info.get("pid") == os.getpid() or not _alive(int(info.get("pid", -1))):
        return None
    return info


def import_published(info: dict) -> Optional[List[HbmBuffer]]:
    out = []
    for hx in info["handles"]:
        raw = bytes.fromhex(hx)
        p = ctypes.c_void_p(0)
        err = _kern().dw_ipc_open_handle(raw, ctypes.byref(p))
        if err != 0:
            logger.warning(f"importing the standby's HBM staging failed ({err}); keeping local buffers")
            for b in out:
                b.release()
            return None
        out.append(HbmBuffer(int(p.value), int(info["nbytes"]), int(info["pid"]), owned=False))
    return out
