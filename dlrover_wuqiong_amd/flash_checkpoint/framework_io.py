"""Capture a training framework's ``torch.save`` / ``torch.load`` calls.

Megatron-LM and DeepSpeed write checkpoints with plain ``torch.save(obj,
path)`` inside their own ``save_checkpoint``.  Flash checkpointing keeps
their on-disk layout (so their own loaders, converters and tooling keep
working) by swapping ``torch.save`` while the framework's save runs: every
``(path, state dict)`` it would have written is captured, the captured state
is snapshotted into shared memory by the flash engine, and the agent later
writes exactly those paths.  Loading swaps ``torch.load`` so the framework
reads the in-memory copy when one exists.

Parity: reference ``flash_checkpoint/megatron.py:75-108`` and
``deepspeed.py:45-96`` (``MegatronCheckpointer.save/load``,
``AsyncCheckpointAgent.save/load``).
"""

import os
import threading
from contextlib import contextmanager
from typing import Callable, Dict, Optional

import torch

_native_save = torch.save
_native_load = torch.load
_swap_lock = threading.Lock()


class TorchIOInterceptor:
    """``classify(path) -> name`` maps a file path to a state category
    (``model_states`` / ``optim_states`` / file name); ``None`` means write
    through to storage immediately."""

    def __init__(self, classify: Callable[[str], Optional[str]], storage=None):
        self.classify = classify
        self.storage = storage
        self.state_dict: Dict[str, object] = {}
        self.paths: Dict[str, str] = {}
        self.memory_state: Dict[str, object] = {}

    def reset(self):
        self.state_dict = {}
        self.paths = {}

    def save(self, obj, f, *args, **kwargs):
        if not isinstance(f, (str, os.PathLike)):
            return _native_save(obj, f, *args, **kwargs)
        path = os.fspath(f)
        name = self.classify(path)
        if name is None:
            return _native_save(obj, f, *args, **kwargs)
        self.state_dict[name] = obj
        self.paths[name] = path
        return None

    def load(self, f, *args, **kwargs):
        if isinstance(f, (str, os.PathLike)):
            path = os.fspath(f)
            name = self.classify(path)
            if name is not None and name in self.memory_state:
                return self.memory_state[name]
            kwargs.setdefault("map_location", "cpu")
        return _native_load(f, *args, **kwargs)

    @contextmanager
    def capturing(self):
        with _swap_lock:
            torch.save = self.save
            try:
                yield self
            finally:
                torch.save = _native_save

    @contextmanager
    def serving(self, memory_state: Dict[str, object]):
        self.memory_state = memory_state or {}
        with _swap_lock:
            torch.load = self.load
            try:
                yield self
            finally:
                torch.load = _native_load
                self.memory_state = {}


def tag_to_step(tag) -> int:
    """DeepSpeed tags are free-form ("global_step100"); flash checkpoint
    steps are integers: use the trailing number."""
    if isinstance(tag, int):
        return tag
    s = str(tag)
    digits = ""
    for ch in reversed(s):
        if ch.isdigit():
            digits = ch + digits
        elif digits:
            break
    if not digits:
        raise ValueError(f"checkpoint tag {tag!r} carries no step number")
    return int(digits)
