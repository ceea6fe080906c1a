"""Selective activation offloading: keep chosen saved activations in pinned
host memory between forward and backward instead of HBM (or recompute).

    with OffloadActivations(min_bytes=8 << 20, op_filter=lambda t: t.dim() >= 2):
        loss = model(x)          # large saved tensors stream D2H on a side stream
    loss.backward()              # ... and come back H2D just before use

Built on ``torch.autograd.graph.saved_tensors_hooks``: the pack hook copies
a saved tensor into a pinned host buffer on a dedicated HIP copy stream
(ordered after the producing kernel by an event, so forward compute is not
blocked), the unpack hook issues the H2D on the same side stream and makes
the compute stream wait for it.  ``max_inflight`` bounds how many D2H copies
may be pending (copy engines / host PCIe are shared by the GPUs of a node --
the reference's ``index_to_offload`` balancing).  With 288 GB of HBM per
MI355X this is for very long sequences or very large micro-batches; pinned
buffers are recycled across steps by size class.

Parity: ATorch ``atorch/auto/opt_lib/selective_offloading_checkpoint.py``
(``OffloadOpManager``: offload chosen matmul activations to CPU, reload in
backward, free-event queue bounding in-flight copies).
"""

import collections
from typing import Callable, Deque, Dict, List, Optional

import torch


class _PinnedPool:
    def __init__(self):
        self._free: Dict[tuple, List[torch.Tensor]] = collections.defaultdict(list)

    def get(self, shape, dtype) -> torch.Tensor:
        key = (tuple(shape), dtype)
        lst = self._free[key]
        if lst:
            return lst.pop()
        return torch.empty(shape, dtype=dtype, pin_memory=torch.cuda.is_available())

    def put(self, t: torch.Tensor):
        self._free[(tuple(t.shape), t.dtype)].append(t)


class OffloadActivations:
    def __init__(self, min_bytes: int = 1 << 20, op_filter: Optional[Callable[[torch.Tensor], bool]] = None,
                 max_inflight: int = 4, pool: Optional[_PinnedPool] = None):
        self.min_bytes = min_bytes
        self.op_filter = op_filter
        self.max_inflight = max_inflight
        self.pool = pool or _PinnedPool()
        self.offloaded_bytes = 0
        self._inflight: Deque = collections.deque()
        self._to_free: List = []  # (event, host buffer) awaiting H2D completion
        self._stream = None
        self._ctx = None

    def _want(self, t: torch.Tensor) -> bool:
        if not isinstance(t, torch.Tensor) or t.is_sparse or t.device.type != ("cuda" if torch.cuda.is_available()
                                                                                else "cpu"):
            return False
        if isinstance(t, torch.nn.Parameter) or t.numel() * t.element_size() < self.min_bytes:
            return False
        return self.op_filter is None or self.op_filter(t)

    def _reclaim(self):
        keep = []
        for ev, host in self._to_free:
            if ev.query():
                self.pool.put(host)
            else:
                keep.append((ev, host))
        self._to_free = keep

    def _pack(self, t: torch.Tensor):
        if not self._want(t):
            return t
        self._reclaim()
        cuda = t.is_cuda
        host = self.pool.get(t.shape, t.dtype)
        src = t.contiguous() if not t.is_contiguous() else t
        if cuda:
            if self._stream is None:
                self._stream = torch.cuda.Stream(t.device)
            while len(self._inflight) >= self.max_inflight:
                self._inflight.popleft().synchronize()
            self._stream.wait_stream(torch.cuda.current_stream(t.device))
            with torch.cuda.stream(self._stream):
                host.copy_(src, non_blocking=True)
                src.record_stream(self._stream)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            self._inflight.append(ev)
        else:
            host.copy_(src)
            ev = None
        self.offloaded_bytes += t.numel() * t.element_size()
        return ("dwamd_offload", host, t.device, ev, t.stride() if t.is_contiguous() else None)

    def _unpack(self, packed):
        if not (isinstance(packed, tuple) and len(packed) == 5 and packed[0] == "dwamd_offload"):
            return packed
        _, host, device, ev, _stride = packed
        if device.type != "cuda":
            return host
        cur = torch.cuda.current_stream(device)
        with torch.cuda.stream(self._stream):
            if ev is not None:
                self._stream.wait_event(ev)
            out = torch.empty(host.shape, dtype=host.dtype, device=device)
            out.copy_(host, non_blocking=True)
            done = torch.cuda.Event()
            done.record(self._stream)
        cur.wait_event(done)
        out.record_stream(cur)
        self._to_free.append((done, host))  # recycled once the H2D has completed
        return out

    def __enter__(self):
        self._ctx = torch.autograd.graph.saved_tensors_hooks(self._pack, self._unpack)
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        self._ctx.__exit__(*exc)
        self._ctx = None
        return False


class OffloadCheckpointWrapper(torch.nn.Module):
    """Wrap a block so its saved activations are offloaded (the
    ``offload_checkpoint`` counterpart of activation checkpointing)."""

    def __init__(self, module: torch.nn.Module, min_bytes: int = 1 << 20, pool: Optional[_PinnedPool] = None):
        super().__init__()
        self.module = module
        self.min_bytes = min_bytes
        self.pool = pool or _PinnedPool()

    def forward(self, *args, **kwargs):
        if not torch.is_grad_enabled():
            return self.module(*args, **kwargs)
        with OffloadActivations(self.min_bytes, pool=self.pool):
            return self.module(*args, **kwargs)


def apply_offload_checkpoint(model: torch.nn.Module, classes, min_bytes: int = 1 << 20) -> int:
    """Replace every child module of one of ``classes`` by an
    ``OffloadCheckpointWrapper`` (shared pinned pool); returns the count."""
    pool = _PinnedPool()
    n = 0
    for parent in list(model.modules()):
        for name, child in list(parent.named_children()):
            if isinstance(child, tuple(classes)) and not isinstance(parent, OffloadCheckpointWrapper):
                setattr(parent, name, OffloadCheckpointWrapper(child, min_bytes, pool))
                n += 1
    return n
