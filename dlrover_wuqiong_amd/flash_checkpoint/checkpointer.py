"""User-facing checkpointer API (reference
``dlrover/trainer/torch/flash_checkpoint/checkpointer.py:18-65``)."""

from abc import ABC, abstractmethod
from enum import Enum, auto


class StorageType(Enum):
    MEMORY = auto()
    DISK = auto()


class Checkpointer(ABC):
    """Save to host memory in (sub)seconds, persist asynchronously, and on
    load prefer the in-memory copy when every rank has the same step."""

    @abstractmethod
    def save_checkpoint(self, step, state_dict, path, storage_type=StorageType.DISK):
        ...

    @abstractmethod
    def load_checkpoint(self, resuming_path=None):
        ...
