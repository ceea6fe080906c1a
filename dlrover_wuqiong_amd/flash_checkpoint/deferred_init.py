"""Skip a model's random initialisation when a restart restores it anyway.

An import-mode replacement (``dwamd-run --standby-mode import``, the
reference's restart semantics) runs the training script from the top: it
builds the model -- a few hundred ``torch.nn.init`` kernels and their Python
dispatch for GPT2-1.5B (~0.1 s of the restart) -- and the flash-checkpoint
restore then overwrites every parameter.  Around the model constructor::

    with deferred_init() as di:
        model = GPT2(cfg)
    ...
    if ckpt.load_checkpoint(...) is empty:      # nothing was restored
        di.replay()

on a restart (``TORCHELASTIC_RESTART_COUNT`` > 0) the ``torch.nn.init``
functions only record their calls (and the cyclic collector stays off until
the restore or ``discard()`` / ``replay()``); ``replay()`` runs them later, in order,
against the same Parameter objects (so it also reaches storage that
``FlatParams`` / ``.to()`` re-pointed them to).  Outside a restart, or with
``DWAMD_DEFER_INIT=0``, the context is a no-op and ``replay()`` does nothing.

Parity: ATorch's meta-device / ``param_init_fn`` deferred initialisation
(``utils/fsdp_init_util.py``) applied to the restart path of the elastic
agent (reference ``dlrover/python/elastic_agent/torch/training.py``).
"""

import contextlib
import gc
import os
from typing import Callable, List, Tuple

import torch
import torch.nn.init as _init

_FNS = ("uniform_", "normal_", "trunc_normal_", "constant_", "ones_", "zeros_", "eye_", "dirac_",
        "xavier_uniform_", "xavier_normal_", "kaiming_uniform_", "kaiming_normal_", "orthogonal_", "sparse_")


_GC_HELD = False


def hold_gc():
    """Keep the cyclic collector off through a restart's model build and
    restore (a generation-2 pass over a model's worth of fresh objects cost
    80-90 ms at random points of the build, profiles/r4 bench runs)."""
    global _GC_HELD
    if not _GC_HELD and gc.isenabled():
        gc.disable()
        _GC_HELD = True


def release_gc():
    """End :func:`hold_gc`: freeze what is alive now (model, optimizer,
    restored state -- long-lived) out of later full collections, re-enable."""
    global _GC_HELD
    if _GC_HELD:
        _GC_HELD = False
        gc.freeze()
        gc.enable()


def restarting() -> bool:
    try:
        return int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0
    except ValueError:
        return False


class DeferredInit:
    def __init__(self, active: bool):
        self.active = active
        self.calls: List[Tuple[Callable, torch.Tensor, tuple, dict]] = []
        self.replayed = False

    def replay(self) -> int:
        """Run the recorded initialisers (once).  Returns how many ran."""
        if self.replayed or not self.calls:
            release_gc()
            return 0
        self.replayed = True
        with torch.no_grad():
            for fn, t, args, kwargs in self.calls:
                fn(t, *args, **kwargs)
        n = len(self.calls)
        self.calls = []
        release_gc()
        return n

    def discard(self):
        """The restore covered every parameter: drop the recorded calls."""
        self.calls = []
        release_gc()


@contextlib.contextmanager
def deferred_init(active: bool = None):
    """Record instead of run ``torch.nn.init`` calls on a restart (see the
    module docstring); yields a :class:`DeferredInit`."""
    if active is None:
        active = restarting() and os.environ.get("DWAMD_DEFER_INIT", "1") != "0"
    d = DeferredInit(active)
    if not active:
        yield d
        return
    hold_gc()  # released by discard() / replay() or by the checkpoint restore
    saved = {}
    for name in _FNS:
        fn = getattr(_init, name, None)
        if fn is None:
            continue
        saved[name] = fn

        def rec(t, *args, _fn=fn, **kwargs):
            d.calls.append((_fn, t, args, kwargs))
            return t

        setattr(_init, name, rec)
    try:
        yield d
    finally:
        for name, fn in saved.items():
            setattr(_init, name, fn)
