"""Build + load the in-tree native libraries.

Two shared objects are produced next to this file:

* ``libdw_runtime.so`` – host C++ (shm segments, robust process-shared
  lock/queue/dict, parallel file IO, crc32c).  No GPU dependency.
* ``libdw_kernels.so`` – HIP kernels for gfx950 (MFMA/LDS-tiled hot ops,
  flash-checkpoint pack/unpack, fused optimizers) plus host helpers
  (pinned-host registration, async copies on side streams).

Both are plain C ABI libraries loaded with :mod:`ctypes`; PyTorch tensors are
passed as raw device pointers and the current HIP stream handle, so the
kernels run on PyTorch's stream (and are captured by hipGraphs) without any
PyTorch C++ ABI coupling.  ``torch`` is always imported first so that the HIP
runtime already mapped by PyTorch (soname ``libamdhip64.so.7``) is the one our
library binds to - a second runtime instance would not share streams.
"""

import ctypes
import os
import threading

from .build import build_kernels, build_runtime, kernels_lib_path, runtime_lib_path

_lock = threading.Lock()
_runtime = None
_kernels = None


class NativeLibraryError(RuntimeError):
    pass


def runtime():
    """The host runtime library (always available; built on demand)."""
    global _runtime
    if _runtime is not None:
        return _runtime
    with _lock:
        if _runtime is None:
            path = runtime_lib_path()
            if not os.path.exists(path) or _stale(path, "runtime"):
                build_runtime()
            lib = ctypes.CDLL(path)
            _declare_runtime(lib)
            _runtime = lib
    return _runtime


def kernels(required: bool = True):
    """The HIP kernel library.

    On a GPU host this must load: ops fail loudly rather than silently running
    an eager fallback (``required=True``).
    """
    global _kernels
    if _kernels is not None:
        return _kernels
    with _lock:
        if _kernels is None:
            import torch  # noqa: F401  (bind to the HIP runtime torch loaded)

            path = kernels_lib_path()
            ab = os.environ.get("DWAMD_KERNELS_LIB_AB", "")  # A/B runs only (scripts/build_variant_lib.py)
            if ab:
                path = ab
            elif not os.path.exists(path) or _stale(path, "kernels"):
                try:
                    build_kernels()
                except Exception as e:  # pragma: no cover - depends on toolchain
                    if required:
                        raise NativeLibraryError(f"cannot build HIP kernels: {e}") from e
                    return None
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            from . import kernel_sigs

            kernel_sigs.declare(lib)
            _kernels = lib
    return _kernels


def _stale(lib_path: str, which: str) -> bool:
    if os.environ.get("DWAMD_NO_REBUILD", "0") == "1":
        return False
    from .build import sources_digest, sources_for

    try:
        lib_m = os.path.getmtime(lib_path)
    except OSError:
        return True
    try:
        with open(lib_path + ".srcsha") as f:
            return f.read().strip() != sources_digest(which)  # content decides when recorded
    except OSError:
        pass
    for s in sources_for(which):
        try:
            if os.path.getmtime(s) > lib_m:
                return True
        except OSError:
            pass
    return False


def _declare_runtime(lib):
    c = ctypes
    vp, u64, i64, i32, u32, dbl, cp = (
        c.c_void_p, c.c_uint64, c.c_int64, c.c_int, c.c_uint32, c.c_double, c.c_char_p)
    sig = {
        "dw_last_error": (cp, []),
        "dw_shm_create": (vp, [cp, u64, i32]),
        "dw_shm_open": (vp, [cp, c.POINTER(u64)]),
        "dw_shm_exists": (i32, [cp]),
        "dw_shm_size": (i64, [cp]),
        "dw_shm_close": (i32, [vp, u64]),
        "dw_shm_unlink": (i32, [cp]),
        "dw_prefault": (i32, [vp, u64, i32]),
        "dw_memcpy_parallel": (i32, [vp, vp, u64, i32]),
        "dw_write_file": (i32, [cp, vp, u64, u64, i32, i32]),
        "dw_read_file": (i32, [cp, vp, u64, u64, i32]),
        "dw_read_file_direct": (i32, [cp, vp, u64, u64, i32, i32]),
        "dw_crc32c": (u32, [vp, u64, u32]),
        "dw_ctl_open": (vp, [cp, i32, u32, u64, u64]),
        "dw_ctl_close": (i32, [vp]),
        "dw_lock_acquire": (i32, [vp, i32, dbl]),
        "dw_lock_release": (i32, [vp]),
        "dw_lock_locked": (i32, [vp]),
        "dw_queue_put": (i32, [vp, vp, u64, i32, dbl]),
        "dw_queue_get": (i64, [vp, vp, u64, i32, dbl, c.POINTER(u64)]),
        "dw_queue_size": (i64, [vp]),
        "dw_blob_set": (i32, [vp, vp, u64]),
        "dw_blob_get": (i64, [vp, vp, u64, c.POINTER(u64), c.POINTER(u64)]),
        "dw_blob_version": (u64, [vp]),
        "dw_runtime_abi_version": (i32, []),
        "dw_ring_open": (vp, [cp, i32, u32, u64, u32, u32, u32, dbl]),
        "dw_ring_close": (i32, [vp]),
        "dw_ring_slot_bytes": (u64, [vp]),
        "dw_ring_nslots": (u32, [vp]),
        "dw_ring_epoch": (u32, [vp]),
        "dw_ring_base": (vp, [vp]),
        "dw_ring_total": (u64, [vp]),
        "dw_ring_slot": (vp, [vp, i64]),
        "dw_ring_write_acquire": (i64, [vp, dbl]),
        "dw_ring_write_commit": (i32, [vp, i64, u64]),
        "dw_ring_read_acquire": (i64, [vp, i32, dbl, c.POINTER(u64)]),
        "dw_ring_read_release": (i32, [vp, i32, i64]),
        "dw_ring_stop": (i32, [vp]),
        "dw_ring_abort": (i32, [vp]),
        "dw_ring_next_epoch": (i32, [vp, dbl]),
        "dw_ring_wait_epoch": (i32, [vp, u32, dbl]),
        "dw_cpu_adamw": (i32, [vp, vp, i32, vp, vp, vp, u64, c.c_float, c.c_float, c.c_float, c.c_float,
                               c.c_float, c.c_float, c.c_float, c.c_float, i32]),
        "dw_cpu_sumsq": (dbl, [vp, i32, u64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def last_error() -> str:
    return runtime().dw_last_error().decode(errors="replace")
