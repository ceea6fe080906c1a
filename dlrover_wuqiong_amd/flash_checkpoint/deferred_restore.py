"""Optimizer state restored behind the first training step.

A restart's flash-checkpoint restore from host shm is PCIe-bound (GPT2-1.5B:
21.8 GB at ~57 GB/s, 0.38 s of device time), and 86 % of those bytes are
optimizer state (fp32 master weights, exp_avg, exp_avg_sq) that nothing
reads until the optimizer update at the END of the first step.  The engine
therefore copies the model (and every non-optimizer leaf) on the compute
stream as before, and the leaves under an ``optim*`` / ``opt`` key (first two
levels) of the checkpointed dict on a side stream; the restore returns once
they are enqueued, and the first forward / backward runs while those DMAs
land (SDMA engines, no CU time).  A ``torch.cuda.synchronize()`` after the
load still waits for everything.

Ordering is enforced on the device, never by host waits:
  * every ``torch.optim.Optimizer.step`` (a global step pre-hook, installed
    with the first deferred restore; this package's flat optimizers are
    ``torch.optim.Optimizer`` subclasses) makes the current stream wait for
    the deferred copies;
  * flash-checkpoint snapshots order their copy stream after them
    (``copier._pending_updates``), restores join them;
  * :func:`wait_all` for any other reader of optimizer state.

``DWAMD_DEFER_OPTIM_RESTORE=0`` restores everything on the compute stream.
The time until the whole state is resident is still measured
(:meth:`DeferredRestore.resident_sec`) and is what ``bench.py`` reports as
``load_sec``; the gain shows up as recovery time (the first step overlaps the
copies).

Parity: the reference restores the whole state dict synchronously before
training resumes (``dlrover/trainer/torch/flash_checkpoint/engine.py``
``load``); this is an MI355X-side overlap of the same restore.
"""

import os
import threading
import time
from typing import Callable, List, Optional

import torch

_PENDING: List["DeferredRestore"] = []
_LOCK = threading.Lock()
_HOOK = None


def enabled() -> bool:
    return os.environ.get("DWAMD_DEFER_OPTIM_RESTORE", "1") != "0"


def is_deferred_key(key) -> bool:
    """Top-level checkpoint keys whose tensors may land after the restore
    call returns: optimizer state."""
    return isinstance(key, str) and ("optim" in key.lower() or key.lower() == "opt")


class DeferredRestore:
    """Copies enqueued (by the calling thread, before the restore returns:
    a ``torch.cuda.synchronize()`` after the load still covers them) on
    ``stream`` after ``ready`` (an event of the compute stream); ``event``
    completes when they landed.  A helper thread only waits for that to
    time the residency."""

    def __init__(self, device, stream, ready, enqueue: Callable[[object], None], t0: float):
        self.device = device
        self.stream = stream
        self.t0 = t0
        self.done_at: Optional[float] = None
        with torch.cuda.device(device):
            stream.wait_event(ready)
            enqueue(stream)
            self.event = stream.record_event()
        self.enqueued_at = time.perf_counter()
        self._thread = threading.Thread(target=self._time, daemon=True, name="dwamd-deferred-restore")
        self._thread.start()

    def _time(self):
        self.event.synchronize()
        self.done_at = time.perf_counter()

    def wait(self, stream=None):
        """Order ``stream`` (default: current) after the copies (device-side
        wait, the host does not block)."""
        (stream or torch.cuda.current_stream(self.device)).wait_event(self.event)

    def ready_event(self):
        return self.event

    @property
    def complete(self) -> bool:
        return self.done_at is not None or self.event.query()

    def resident_sec(self, timeout: Optional[float] = None) -> Optional[float]:
        """Seconds from the restore call until every deferred byte landed
        (blocks until then)."""
        self._thread.join(timeout)
        return None if self.done_at is None else self.done_at - self.t0


class _Extra:
    """A plain event registered like a deferred restore (e.g. verification
    reads that must precede the first optimizer update)."""

    def __init__(self, device, event):
        self.device, self.event = device, event

    def wait(self, stream=None):
        (stream or torch.cuda.current_stream(self.device)).wait_event(self.event)

    def ready_event(self):
        return self.event

    @property
    def complete(self) -> bool:
        return self.event.query()


def add(d):
    with _LOCK:
        _PENDING.append(d)
    _install_hook()


def add_event(event, device=None):
    add(_Extra(torch.device("cuda", torch.cuda.current_device()) if device is None else device, event))


def pending(device=None) -> list:
    with _LOCK:
        _PENDING[:] = [d for d in _PENDING if not d.complete]
        out = list(_PENDING)
    if device is not None:
        dev = torch.device(device)
        out = [d for d in out if torch.device(d.device) == dev]
    return out


def events(device=None) -> list:
    """Completion events of the pending deferred copies (for streams that
    must order after them)."""
    return [d.ready_event() for d in pending(device)]


def wait_all(stream=None, device=None):
    for d in pending(device):
        d.wait(stream)


def synchronize_all(device=None):
    """Host-side wait until every pending deferred copy landed: before the
    host memory they read (pinned shm) is unregistered or unmapped."""
    for d in pending(device):
        d.event.synchronize()


def _step_pre_hook(optimizer, args, kwargs):
    if _PENDING:
        wait_all()


def _install_hook():
    global _HOOK
    if _HOOK is None:
        from torch.optim.optimizer import register_optimizer_step_pre_hook

        _HOOK = register_optimizer_step_pre_hook(_step_pre_hook)
