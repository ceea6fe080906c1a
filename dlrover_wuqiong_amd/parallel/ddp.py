"""Data parallelism over flat gradient buckets (RCCL over xGMI).

Gradients live in one flat buffer (``FlatParams``); a bucket is a contiguous
slice of it.  A post-accumulate-grad hook counts ready parameters per bucket
and launches ``all_reduce`` on the slice as soon as the bucket is complete,
so communication overlaps the rest of backward (RCCL runs on its own stream;
``work.wait()`` only makes the compute stream wait, never the host).

Bucket sizing for MI355X: an 8-GPU node is a fully connected xGMI mesh
(7 links x ~153 GB/s per GPU); ring all-reduce is per-link bound, so a few
large buckets (default 128 MiB) amortise the per-collective latency while
still leaving several buckets to overlap with backward.

Readiness is counted, not assumed: the first synchronised backward only
records how many times each parameter's hook fires (PyTorch fires the
post-accumulate hook once per backward even for the fused ops that write the
flat gradient themselves and return ``None``; a parameter shared by two ops
fires twice) and reduces every bucket at ``finish_gradient_sync``.  Later
backwards launch a bucket when all of its recorded hook calls have arrived.
Buckets holding a parameter that was unused in the calibration pass are never
launched early (an MoE expert may get tokens later), and a gradient arriving
for an already-launched bucket raises instead of being silently dropped.

Gradients are SUMMED; the optimizer divides by the world size inside its
fused update (``grad_scale``), in fp32, instead of a separate scaling pass.

``grad_comm_bits=8`` (or 4) reduces each bucket through the quantized
collectives instead (``quantized_comm.quantized_all_reduce``: int8 / int4
all-to-all reduce-scatter + all-gather, ~1/2 (1/4) of bf16's wire bytes)
for bandwidth-starved links (multi-node RDMA); it runs on a side stream so
it still overlaps the rest of backward.  Lossy: ~2^-(bits-1) of each
group's absmax per element.  Within one xGMI node the exact bf16 all-reduce
is the default.

Parity: reference trainers wrap models in torch DDP
(dlrover/trainer/torch/elastic/trainer.py, atorch data_parallel/*); this is
the framework's own replacement tuned for flat buffers.
"""

from contextlib import contextmanager
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .flat import FlatParams


class FlatDDP(nn.Module):
    def __init__(self, module: nn.Module, flat: FlatParams, process_group=None, bucket_mb: int = 128,
                 broadcast_params: bool = True, grad_comm_bits: Optional[int] = None):
        super().__init__()
        self.module = module
        self.flat = flat
        self.pg = process_group
        if grad_comm_bits not in (None, 4, 8):
            raise ValueError("grad_comm_bits must be None, 8 or 4")
        self.grad_comm_bits = grad_comm_bits
        self._side = None
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.buckets = flat.grad_slices(bucket_mb << 20)
        self._bucket_of = {}
        for bi, (_s, _e, idxs) in enumerate(self.buckets):
            for i in idxs:
                self._bucket_of[i] = bi
        self._pending: List[int] = []
        self._works: List[Optional[object]] = []
        self._sync = True
        self._expected: Optional[List[int]] = None  # hook calls per parameter per backward
        self._calls = [0] * len(flat.params)
        self._reset()
        if self.world > 1:
            if broadcast_params:
                dist.broadcast(flat.data, src=self._global_src(), group=process_group)
            for i, p in enumerate(flat.params):
                p.register_post_accumulate_grad_hook(self._make_hook(i))

    def _global_src(self):
        if self.pg is None:
            return 0
        return dist.get_global_rank(self.pg, 0)

    def _reset(self):
        self._calls = [0] * len(self.flat.params)
        self._works = [None] * len(self.buckets)
        if self._expected is None:
            self._pending = [-1] * len(self.buckets)  # calibration pass: never launch early
            return
        self._pending = []
        for (_s, _e, idxs) in self.buckets:
            exp = [self._expected[i] for i in idxs]
            self._pending.append(sum(exp) if all(exp) else -1)

    def _make_hook(self, idx):
        def hook(_p):
            if not self._sync:
                return
            self._calls[idx] += 1
            b = self._bucket_of[idx]
            if self._works[b] is not None:
                raise RuntimeError(
                    f"FlatDDP: gradient of parameter {idx} arrived after its bucket {b} was reduced "
                    "(the parameter is used more often than in the first backward)")
            if self._pending[b] > 0:
                self._pending[b] -= 1
                if self._pending[b] == 0:
                    self._works[b] = self._reduce(b)
        return hook

    def _reduce(self, b):
        s, e, _ = self.buckets[b]
        g = self.flat.grad[s:e]
        if self.grad_comm_bits is None:
            return dist.all_reduce(g, group=self.pg, async_op=True)
        from .quantized_comm import quantized_all_reduce

        if not g.is_cuda:
            quantized_all_reduce(g, self.pg, bits=self.grad_comm_bits)
            return _Done()
        # quantize -> all-to-all -> dequant-reduce -> quantize -> all-gather ->
        # dequantize on a side stream, ordered after the gradient's producer
        if self._side is None:
            self._side = torch.cuda.Stream(device=g.device)
        ready = torch.cuda.current_stream(g.device).record_event()
        with torch.cuda.stream(self._side):
            self._side.wait_event(ready)
            quantized_all_reduce(g, self.pg, bits=self.grad_comm_bits)
            done = self._side.record_event()
        g.record_stream(self._side)
        return _StreamDone(done)

    def forward(self, *args, **kwargs):
        self._reset()
        return self.module(*args, **kwargs)

    @contextmanager
    def no_sync(self):
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def finish_gradient_sync(self):
        """Wait for every bucket (launching any that never completed, e.g.
        buckets holding unused parameters)."""
        if self.world <= 1:
            return
        self.flat.finalize_grads()  # lazily zeroed grads nobody wrote (the backward-end callback did it already)
        if self._expected is None:
            self._expected = list(self._calls)
        for b in range(len(self.buckets)):
            if self._works[b] is None:
                self._works[b] = self._reduce(b)
        for w in self._works:
            w.wait()
        self._reset()


class _Done:
    def wait(self):
        return True


class _StreamDone:
    """The compute stream waits for the side-stream reduction (no host sync)."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True
