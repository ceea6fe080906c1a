"""Batch serialization into the native shared-memory ring (``csrc/runtime/
dw_ring.cpp``).

A slot holds one batch: ``[u32 header_len][JSON header][pad to 64 B][tensor
bytes, each 64 B aligned]``.  The header carries the pytree spec of the batch
(``torch.utils._pytree.treespec_dumps``), the non-tensor leaves and, per
tensor, ``(dtype, shape, offset)`` -- no pickle anywhere, so a reader never
executes anything a writer produced.

Readers either copy a batch out to CPU tensors, or, with ``device="cuda"``,
issue the host->device copies straight from the slot: the whole ring is
registered once with ``hipHostRegister`` so the DMA engine reads the shm
pages directly (no staging copy), on a side stream; the slot is released
once that copy's event has completed.
"""

import ctypes
import json
import struct
from typing import Any, List, Optional, Tuple

import torch
import torch.utils._pytree as pytree

from ..._native import runtime

SHARED, BROADCAST = 0, 1
_ALIGN = 64
_DTYPES = {str(d).replace("torch.", ""): d for d in (
    torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.int16,
    torch.int8, torch.uint8, torch.bool)}


class RingTimeout(TimeoutError):
    pass


def _al(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def encode_header(batch) -> Tuple[bytes, List[torch.Tensor], int]:
    """-> (JSON header, tensors, total bytes).  Tensor offsets in the header
    are relative to the data start ``_al(4 + len(header))``."""
    leaves, spec = pytree.tree_flatten(batch)
    tensors, metas, plain = [], [], []
    off = 0
    for i, x in enumerate(leaves):
        if isinstance(x, torch.Tensor):
            t = x.detach()
            if t.is_cuda:
                t = t.cpu()
            t = t.contiguous()
            tensors.append(t)
            metas.append([i, str(t.dtype).replace("torch.", ""), list(t.shape), off])
            off = _al(off + t.numel() * t.element_size())
        else:
            plain.append([i, x])
    raw = json.dumps({"spec": pytree.treespec_dumps(spec), "n": len(leaves), "t": metas, "p": plain}).encode()
    return raw, tensors, _al(4 + len(raw)) + off


def batch_nbytes(batch) -> int:
    return encode_header(batch)[2]


class ShmBatchRing:
    """One ring endpoint.  ``create=True`` on the producer that owns it."""

    def __init__(self, name: str, create: bool, nslots: int = 8, slot_bytes: int = 1 << 20, nreaders: int = 1,
                 mode: int = SHARED, nproducers: int = 1, timeout: float = 300.0):
        self.lib = runtime()
        self.name = name
        self.create = create
        self.h = self.lib.dw_ring_open(name.encode(), int(create), nslots, slot_bytes, nreaders, mode, nproducers,
                                       float(timeout))
        if not self.h:
            raise RingTimeout(f"cannot {'create' if create else 'attach'} shm ring {name}")
        self.slot_bytes = self.lib.dw_ring_slot_bytes(self.h)
        self._registered = False
        self._copy_stream = None
        self._pending: Optional[Tuple[int, int, Any]] = None  # (reader, ticket, event)

    # ------------------------------------------------------------- write
    def put(self, batch, timeout: float = 30.0) -> bool:
        """Serialize ``batch`` into the next free slot.  False if the epoch was
        stopped (abort)."""
        raw, tensors, total = encode_header(batch)
        if total > self.slot_bytes:
            raise ValueError(f"batch of {total} B exceeds the ring slot size {self.slot_bytes} B")
        t = self.lib.dw_ring_write_acquire(self.h, float(timeout))
        if t == -3:
            return False
        if t < 0:
            raise RingTimeout(f"ring {self.name}: no free slot within {timeout}s (readers stalled?)")
        base = self.lib.dw_ring_slot(self.h, t)
        ctypes.memmove(base, struct.pack("<I", len(raw)), 4)
        ctypes.memmove(base + 4, raw, len(raw))
        data = base + _al(4 + len(raw))
        for m, x in zip(json.loads(raw)["t"], tensors):
            n = x.numel() * x.element_size()
            if n:
                ctypes.memmove(data + m[3], x.data_ptr(), n)
        self.lib.dw_ring_write_commit(self.h, t, total)
        return True

    def stop(self):
        self.lib.dw_ring_stop(self.h)

    def abort(self):
        self.lib.dw_ring_abort(self.h)

    def next_epoch(self, timeout: float = 300.0):
        if self.lib.dw_ring_next_epoch(self.h, float(timeout)) != 0:
            raise RingTimeout(f"ring {self.name}: readers did not drain the previous epoch")

    def wait_epoch(self, e: int, timeout: float = 300.0):
        if self.lib.dw_ring_wait_epoch(self.h, e, float(timeout)) != 0:
            raise RingTimeout(f"ring {self.name}: epoch {e} not started")

    # -------------------------------------------------------------- read
    def _ensure_registered(self):
        if self._registered:
            return
        from ..._native import kernels

        k = kernels(required=True)
        err = k.dw_host_register(self.lib.dw_ring_base(self.h), self.lib.dw_ring_total(self.h))
        if err != 0:
            raise RuntimeError(f"hipHostRegister of the batch ring failed ({err})")
        self._registered = True
        self._copy_stream = torch.cuda.Stream()

    def _release_pending(self):
        if self._pending is not None:
            reader, ticket, ev = self._pending
            if ev is not None:
                ev.synchronize()
            self.lib.dw_ring_read_release(self.h, reader, ticket)
            self._pending = None

    def get(self, reader: int = 0, timeout: float = 30.0, device: Optional[torch.device] = None):
        """Next batch, or ``None`` at the end of the epoch."""
        self._release_pending()
        nb = ctypes.c_uint64(0)
        t = self.lib.dw_ring_read_acquire(self.h, reader, float(timeout), ctypes.byref(nb))
        if t == -2:
            return None
        if t < 0:
            raise RingTimeout(f"ring {self.name}: no batch within {timeout}s")
        base = self.lib.dw_ring_slot(self.h, t)
        (hlen,) = struct.unpack("<I", ctypes.string_at(base, 4))
        hdr = json.loads(ctypes.string_at(base + 4, hlen))
        base += _al(4 + hlen)  # tensor data start
        leaves: List[Any] = [None] * hdr["n"]
        for i, v in hdr["p"]:
            leaves[i] = v
        gpu = device is not None and torch.device(device).type == "cuda"
        ev = None
        if gpu:
            self._ensure_registered()
            cur = torch.cuda.current_stream(device)
            with torch.cuda.stream(self._copy_stream):
                for i, dt, shape, off in hdr["t"]:
                    dst = torch.empty(shape, dtype=_DTYPES[dt], device=device)
                    n = dst.numel() * dst.element_size()
                    if n:
                        src = (ctypes.c_char * n).from_address(base + off)
                        host = torch.frombuffer(src, dtype=_DTYPES[dt], count=dst.numel()).view(shape)
                        dst.copy_(host, non_blocking=True)
                    dst.record_stream(cur)
                    leaves[i] = dst
                ev = torch.cuda.Event()
                ev.record(self._copy_stream)
            cur.wait_event(ev)
            self._pending = (reader, t, ev)  # released at the next get()
        else:
            for i, dt, shape, off in hdr["t"]:
                dtype = _DTYPES[dt]
                numel = 1
                for s in shape:
                    numel *= s
                n = numel * torch.empty((), dtype=dtype).element_size()
                if n:
                    src = (ctypes.c_char * n).from_address(base + off)
                    leaves[i] = torch.frombuffer(bytearray(src), dtype=dtype, count=numel).view(shape)
                else:
                    leaves[i] = torch.empty(shape, dtype=dtype)
            self.lib.dw_ring_read_release(self.h, reader, t)
        return pytree.tree_unflatten(leaves, pytree.treespec_loads(hdr["spec"]))

    def close(self, unlink: Optional[bool] = None):
        if self.h is None:
            return
        self._release_pending()
        if self._registered:
            from ..._native import kernels

            kernels(required=True).dw_host_unregister(self.lib.dw_ring_base(self.h))
            self._registered = False
        self.lib.dw_ring_close(self.h)
        self.h = None
        if unlink if unlink is not None else self.create:
            self.lib.dw_shm_unlink(self.name.encode())

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
