"""Flat (contiguous) parameter and gradient buffers.

Every trainable parameter of a module is re-pointed to a view of ONE flat
buffer (``param.data``), and its ``.grad`` to a view of ONE flat gradient
buffer.  Consequences, all deliberate for MI355X:

* bucketed gradient all-reduce = contiguous slices of the flat grad buffer
  (no pack/unpack copies before RCCL);
* the optimizer update is one streaming kernel over the whole buffer
  (``optim.hip``), HBM-bound at ~28 B/element;
* a flash checkpoint of model + optimizer state is a handful of long
  contiguous copies (``flash_checkpoint/layout.py`` coalesces by storage).

Parameters are placed in *reverse* registration order so that backward
(which produces gradients roughly from the last layer to the first) fills
the buffer front to back and the first DDP bucket is ready first.  Every
parameter starts on a 64-element boundary; the optimizer's weight-decay mask
has one byte per 64-element block.
"""

import os
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn as nn

ALIGN = 64


def default_no_decay(name: str, p: torch.Tensor) -> bool:
    """GPT/Llama convention: no weight decay on biases, norms, 1-D params."""
    return p.ndim < 2 or name.endswith(".bias") or "norm" in name.lower() or ".ln" in name


class FlatParams:
    def __init__(self, module: nn.Module, dtype: Optional[torch.dtype] = None, device=None,
                 no_decay_fn: Callable[[str, torch.Tensor], bool] = default_no_decay,
                 grad_dtype: Optional[torch.dtype] = None, direct_grads: bool = True,
                 lazy_zero_grad: Optional[bool] = None, named: Optional[List[Tuple[str, nn.Parameter]]] = None,
                 pad_to: int = ALIGN, data: Optional[torch.Tensor] = None, grad: Optional[torch.Tensor] = None):
        """``direct_grads``: the fused ops (``ops/linear.py``, norms, bias
        activations) accumulate straight into the flat ``.grad`` views
        (``ops/_grad.py``); call ``zero_grad()`` (not ``set_to_none``) once
        per optimizer step.  ``lazy_zero_grad`` (training loops that only
        produce gradients by backward; ``DWAMD_LAZY_ZERO_GRAD=0/1``
        overrides): ``zero_grad()`` skips the pass over the buffer and the
        next backward's first contributions overwrite -- gradients read
        between ``zero_grad()`` and the end of the next backward are
        undefined, and gradients written by hand after ``zero_grad()`` need
        the eager default.

        Flat-unit FSDP (``parallel/flat_fsdp.py``) builds one per unit:
        ``named`` (an explicit parameter list, in buffer order) instead of
        the module's, ``pad_to`` (the buffer's numel rounded up to a multiple,
        world x 64 there) and ``data`` / ``grad`` (caller-owned buffers of
        that numel, e.g. a slice of the rank's shard buffer at world 1)."""
        if named is None:
            named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
            # tied weights appear once in named_parameters (dedup by identity)
            named.reverse()
        first = named[0][1] if named else None
        self.dtype = dtype or (first.dtype if first is not None else torch.float32)
        self.grad_dtype = grad_dtype or self.dtype
        self.device = torch.device(device) if device is not None else (
            first.device if first is not None else torch.device("cpu"))
        self.names: List[str] = []
        self.params: List[nn.Parameter] = []
        self.offsets: List[Tuple[int, int]] = []  # (offset, numel)
        off = 0
        for n, p in named:
            self.names.append(n)
            self.params.append(p)
            self.offsets.append((off, p.numel()))
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = (off + pad_to - 1) // pad_to * pad_to
        if data is None:
            data = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        if grad is None:
            grad = torch.zeros(self.numel, dtype=self.grad_dtype, device=self.device)
        if data.numel() != self.numel or grad.numel() != self.numel:
            raise ValueError(f"FlatParams: buffers of {data.numel()} / {grad.numel()} elements, {self.numel} needed")
        self.data, self.grad = data, grad
        mask = torch.ones(max(1, self.numel // ALIGN), dtype=torch.uint8)
        for n, p, (o, c) in zip(self.names, self.params, self.offsets):
            view = self.data[o:o + c].view_as(p)
            with torch.no_grad():
                if not p.is_meta:  # (a meta-device model: the owner fills the buffer, parallel/flat_fsdp.py)
                    view.copy_(p.data.to(self.device, self.dtype))
            p.data = view
            p.grad = self.grad[o:o + c].view_as(p)
            p._dwamd_direct = bool(direct_grads)
            if no_decay_fn(n, p):
                mask[o // ALIGN:(o + c + ALIGN - 1) // ALIGN] = 0
        self.decay_mask = mask.to(self.device)
        self._index: Dict[int, int] = {id(p): i for i, p in enumerate(self.params)}
        # Lazy zeroing (opt-in): zero_grad() only opens a new gradient
        # generation; the first writer of each parameter in it OVERWRITES
        # (GEMMs with beta = 0, reductions without accumulate -- claim()),
        # autograd-accumulated parameters are zeroed by a pre-hook just before
        # their first accumulation, and whatever nobody wrote is zeroed when
        # the backward ends (or before any flat-buffer reader).  Saves the
        # zero pass over the buffer and the C read of every weight-gradient
        # GEMM: 0.5 + 1.3 ms per GPT2-1.5B step (profiles/r4/wgrad_beta_ab.jsonl).
        env = os.environ.get("DWAMD_LAZY_ZERO_GRAD")
        lazy = (env == "1") if env is not None else bool(lazy_zero_grad)
        self.lazy_zero = bool(direct_grads) and lazy
        self._fresh = False  # a generation is open: unwritten grads hold stale values
        self._written: set = set()
        self._finalize_queued = False
        for i, p in enumerate(self.params):
            p._dwamd_flat, p._dwamd_idx = self, i
            if self.lazy_zero:
                p.register_hook(self._make_zero_hook(i))

    # ------------------------------------------------------ lazy gradient zeroing
    def _make_zero_hook(self, i):
        def hook(grad):
            # runs before autograd accumulates ``grad`` into p.grad
            if self._fresh and i not in self._written:
                self.claim(i)
                g = self.params[i].grad
                if g is not None:  # (detached by the user: autograd creates a fresh one)
                    g.zero_()
            return None
        return hook

    def claim(self, i: int) -> bool:
        """The caller is about to write parameter ``i``'s gradient: True if
        it holds nothing of this generation yet (the writer overwrites instead
        of accumulating)."""
        if not self._fresh or i in self._written:
            return False
        self._written.add(i)
        if not self._finalize_queued:
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self.finalize_grads)
                self._finalize_queued = True
            except RuntimeError:
                pass  # outside a backward pass: readers call finalize_grads() themselves
        return True

    def finalize_grads(self):
        """Zero every gradient this generation did not write (unused
        parameters); afterwards the flat gradient is fully defined and later
        backwards accumulate.  Idempotent; cheap when everything was written."""
        self._finalize_queued = False
        if not self._fresh:
            return
        self._fresh = False
        if len(self._written) == len(self.params):
            self._written = set()
            return
        lo = hi = None
        for i, (o, c) in enumerate(self.offsets):
            if i in self._written:
                if lo is not None:
                    self.grad[lo:hi].zero_()
                    lo = None
                continue
            end = o + (c + ALIGN - 1) // ALIGN * ALIGN
            if lo is None:
                lo = o
            hi = end
        if lo is not None:
            self.grad[lo:hi].zero_()
        self._written = set()

    def index_of(self, p) -> int:
        return self._index[id(p)]

    def zero_grad(self):
        if self.lazy_zero:
            # (an overlapped optimizer update still reading them is joined by
            # the next forward before any backward writes)
            self._fresh, self._written, self._finalize_queued = True, set(), False
            return
        ovl = getattr(self, "_step_overlap", None)
        if ovl is not None and ovl.pending:  # an overlapped optimizer update still reads them
            ovl.zero_grad()
            return
        self.grad.zero_()

    def reattach_grads(self):
        """Re-point .grad views (e.g. after someone set grads to None)."""
        for p, (o, c) in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + c].data_ptr():
                p.grad = self.grad[o:o + c].view_as(p)

    def grad_slices(self, bucket_bytes: int) -> List[Tuple[int, int, List[int]]]:
        """Partition [0, numel) into contiguous buckets of ~bucket_bytes
        at parameter boundaries: (start, end, param indices)."""
        esz = self.grad.element_size()
        target = max(1, bucket_bytes // esz)
        buckets = []
        start, idxs = 0, []
        for i, (o, c) in enumerate(self.offsets):
            idxs.append(i)
            end = o + (c + ALIGN - 1) // ALIGN * ALIGN
            if end - start >= target:
                buckets.append((start, end, idxs))
                start, idxs = end, []
        if idxs:
            buckets.append((start, self.numel, idxs))
        return buckets
