"""Optimizer step overlapped with the next forward pass.

The fused AdamW / AGD update (``optim.hip``) is a pure HBM stream at ~28 B
per parameter: 7.7 ms per step for GPT2-1.5B on one MI355X, 6.5 % of the
step, during which the matrix cores idle.  The next step's forward is
GEMM-bound and touches the parameters layer by layer, so the update can run
*under* it:

* ``step()`` computes the clip coefficient on the compute stream (it needs
  every gradient), then enqueues the update in ``chunks`` parameter-aligned
  pieces on a side stream, in FORWARD order (``FlatParams`` stores
  parameters in reverse registration order, so that is back-to-front in the
  buffer), recording an event after each piece;
* a forward pre-hook on every module that owns parameters makes the compute
  stream wait for the event of the last piece holding them -- layer 0 starts
  once its own parameters are updated, while the side stream keeps streaming
  the rest.  A module's parameters must be read inside its own ``__call__``
  (this package's norms route ``add_forward`` through it); a parameter read
  elsewhere is only ordered by the final join;
* ``zero_grad`` during a pending update is enqueued on the side stream after
  the last piece (the update still reads the gradients);
* the top-level forward's post-hook joins the side stream, so the backward
  (which accumulates into the flat gradient) and everything after it are
  ordered after the whole update.

Every element gets exactly the same arithmetic as the one-launch step
(bitwise-identical results, ``tests/test_optim_overlap_gpu.py``).  Readers of
parameters / optimizer state outside a forward must order themselves after
the update: ``join()`` (the flash-checkpoint snapshot does this on its own
copy stream, so the save pause does not wait for the update).

Parity: the reference overlaps nothing here (its optimizer step is a plain
``optimizer.step()`` between iterations, ``atorch/optimizers``); this is an
MI355X-side optimisation of the same update.
"""

import weakref
from typing import Dict, List, Tuple

import torch
import torch.nn as nn

_ACTIVE = weakref.WeakSet()  # StepOverlap objects (for the checkpoint copier)


def pending_events(device=None) -> List["torch.cuda.Event"]:
    """Completion events of every update still pending (for ``device``)."""
    out = []
    for o in list(_ACTIVE):
        if o.pending and (device is None or torch.device(device) == o.device):
            out.append(o.final_event)
    return out


def join_all(stream=None):
    """Order ``stream`` (default: current) after every pending update."""
    for o in list(_ACTIVE):
        if o.pending:
            o.join(stream)


def forward_order_pieces(flat, chunks: int) -> Tuple[List[Tuple[int, int]], Dict[int, int]]:
    """Split the flat buffer at parameter boundaries into ~``chunks`` pieces
    of about equal size, in forward order (parameter index n-1, the first
    registered, first: FlatParams stores them in reverse).  Returns the
    pieces [(lo, hi)] (together exactly [0, numel)) and each parameter
    index's piece."""
    n = len(flat.params)
    target = max(1, flat.numel // max(1, chunks))
    pieces: List[Tuple[int, int]] = []
    piece_of: Dict[int, int] = {}
    hi = flat.numel
    lo = None
    for i in range(n - 1, -1, -1):
        lo = flat.offsets[i][0]
        piece_of[i] = len(pieces)
        if hi - lo >= target:
            pieces.append((lo, hi))
            hi, lo = lo, None
    if lo is not None and hi > lo:
        pieces.append((lo, hi))
    return pieces, piece_of


class StepOverlap:
    def __init__(self, opt, model: nn.Module, chunks: int = 24):
        flat = opt.flat
        if not flat.data.is_cuda:
            raise ValueError("overlapped optimizer step needs a GPU FlatParams")
        self.opt = opt
        self.flat = flat
        self.device = flat.device
        self.side = torch.cuda.Stream(device=self.device)
        pieces, piece_of = forward_order_pieces(flat, chunks)
        self.pieces = pieces
        self.events = [torch.cuda.Event() for _ in pieces]
        self.final_event = torch.cuda.Event()
        self.pending = False
        self._waited = -1
        self._hooks = []
        for m in model.modules():
            own = [p for p in m.parameters(recurse=False) if id(p) in flat._index]
            if not own:
                continue
            need = max(piece_of[flat.index_of(p)] for p in own)
            self._hooks.append(m.register_forward_pre_hook(self._pre_hook(need)))
        self._hooks.append(model.register_forward_hook(lambda *_a: self.join()))
        flat._step_overlap = self
        _ACTIVE.add(self)

    def _pre_hook(self, need: int):
        def hook(_m, _args):
            if self.pending and need > self._waited:
                torch.cuda.current_stream(self.device).wait_event(self.events[need])
                self._waited = need

        return hook

    def launch(self, launch_range):
        """Enqueue ``launch_range(lo, hi)`` (the optimizer's kernel over flat
        elements [lo, hi), issued on the current stream) piece by piece on the
        side stream, after everything the compute stream has enqueued."""
        if self.pending:  # a step without a forward in between: order after it
            self.join()
        cur = torch.cuda.current_stream(self.device)
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            for (lo, hi), ev in zip(self.pieces, self.events):
                launch_range(lo, hi)
                ev.record(self.side)
            self.final_event.record(self.side)
        self._waited = -1
        self.pending = True

    def zero_grad(self):
        """The pending update still reads the gradients: zero them after it."""
        with torch.cuda.stream(self.side):
            self.flat.grad.zero_()
            self.final_event.record(self.side)

    def join(self, stream=None):
        if not self.pending:
            return
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        s.wait_event(self.final_event)
        if stream is None or stream == torch.cuda.current_stream(self.device):
            self.pending = False

    def remove(self):
        self.join()
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.flat._step_overlap = None
        _ACTIVE.discard(self)
