"""Checkpoint storage backends + retention policies.

API parity with reference ``dlrover/python/common/storage.py``
(``CheckpointStorage`` :23-119, ``PosixDiskStorage`` :122, deletion
strategies :190/:219, ``PosixStorageWithDeletion`` :244,
``get_checkpoint_storage`` :321).

Difference: large binary payloads (``write_bytes`` / ``read_into``) go
through the native runtime's multi-threaded pwrite/pread (+fsync), which is
what the agent's persister uses for the raw flash-checkpoint format.
"""

import ctypes
import os
import shutil
from abc import ABC, abstractmethod
from typing import Callable, List, Optional

from .._native import last_error, runtime
from .constants import CheckpointConstant
from .log import logger
from .serialize import ClassMeta


_BIG_WRITE = 4 << 20  # records at least this large go through the native parallel pwrite


def _direct_bit() -> int:
    """``dw_write_file`` mode bit 2: O_DIRECT for the aligned body of large
    records (``DWAMD_PERSIST_ODIRECT=0``: buffered + fsync, page-cache
    write-back)."""
    return 4 if os.environ.get("DWAMD_PERSIST_ODIRECT", "1") == "1" else 0


class _ParallelFileWriter:
    """Sequential-write file object for ``torch.save``.

    ``torch.save`` streams its zip archive through ``write()`` and hands each
    tensor storage over as ONE zero-copy memoryview of the storage bytes (for
    a flash checkpoint: straight out of the shm segment).  Small records
    (pickle, zip headers) are ``os.pwrite``'n; storages go through the native
    runtime's multi-threaded ``pwrite`` at the current offset.  The archive is
    byte-for-byte a regular torch zip file (``torch.load`` reads it)."""

    def __init__(self, path: str, threads: int):
        self.path = path
        self.threads = threads
        self.fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        self.off = 0
        self.big_bytes = 0

    def write(self, b) -> int:
        mv = memoryview(b).cast("B")
        n = mv.nbytes
        if n >= _BIG_WRITE:
            import numpy as np

            addr = np.frombuffer(mv, dtype=np.uint8).ctypes.data
            r = runtime().dw_write_file(self.path.encode(), ctypes.c_void_p(addr), n, self.off, self.threads,
                                        _direct_bit())
            if r != 0:
                raise OSError(f"write {self.path}: {last_error()}")
            self.big_bytes += n
        else:
            done = 0
            while done < n:
                done += os.pwrite(self.fd, mv[done:], self.off + done)
        self.off += n
        return n

    def flush(self):
        pass

    def close(self, fsync: bool = True):
        if self.fd >= 0:
            if fsync:
                os.fsync(self.fd)
            os.close(self.fd)
            self.fd = -1


def fast_torch_save(obj, path: str, threads: int = 16, fsync: bool = True) -> int:
    """``torch.save(obj, path)`` with tensor storages written by parallel
    ``pwrite`` streams, page-aligned records and no CRC pass (the zip CRC is a
    single-threaded ~1 GB/s scan that would dominate a 20+ GB checkpoint;
    ``torch.load`` accepts CRC-less archives).  Returns bytes written."""
    import torch
    from torch.utils.serialization import config

    path = str(path)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    old = (config.save.compute_crc32, config.save.storage_alignment)
    f = _ParallelFileWriter(tmp, threads)
    try:
        config.save.compute_crc32 = False
        config.save.storage_alignment = 4096
        torch.save(obj, f)
        f.close(fsync=fsync)
    except BaseException:
        f.close(fsync=False)
        try:
            os.remove(tmp)
        except OSError:
            pass
        raise
    finally:
        config.save.compute_crc32, config.save.storage_alignment = old
    os.replace(tmp, path)
    return f.off


class CheckpointStorage(ABC):
    @abstractmethod
    def write(self, content, path):
        """Write str/bytes ``content`` to ``path``."""

    @abstractmethod
    def write_state_dict(self, state_dict, path, write_func):
        """Persist a state dict with ``write_func(state_dict, path)``."""

    @abstractmethod
    def read(self, path):
        """Read a text file ('' if absent)."""

    @abstractmethod
    def read_state_dict(self, path, read_func):
        """Read a state dict with ``read_func(path)`` ({} if absent)."""

    @abstractmethod
    def safe_rmtree(self, dir):
        ...

    @abstractmethod
    def safe_remove(self, path):
        ...

    @abstractmethod
    def safe_makedirs(self, dir):
        ...

    @abstractmethod
    def safe_move(self, src_path, dst_path):
        ...

    @abstractmethod
    def commit(self, step: int, success: bool):
        """Called once the checkpoint of ``step`` is (or failed to be) persisted."""

    @abstractmethod
    def exists(self, path: str):
        ...

    @abstractmethod
    def listdir(self, path: str):
        ...

    @abstractmethod
    def get_class_meta(self) -> ClassMeta:
        """How another process rebuilds this storage object."""

    # ------------------------------------------------------------ bulk data
    def write_bytes(self, addr: int, nbytes: int, path: str, offset: int = 0, truncate: bool = True,
                    fsync: bool = True, threads: int = 8):
        """Write ``nbytes`` at host address ``addr`` into ``path``."""
        with open(path, "wb" if truncate else "r+b") as f:
            f.seek(offset)
            f.write((ctypes.c_char * nbytes).from_address(addr))
            if fsync:
                f.flush()
                os.fsync(f.fileno())

    def read_into(self, path: str, addr: int, nbytes: int, offset: int = 0, threads: int = 8):
        with open(path, "rb") as f:
            f.seek(offset)
            f.readinto((ctypes.c_char * nbytes).from_address(addr))


class PosixDiskStorage(CheckpointStorage):
    def write(self, content, path):
        path = str(path)
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        mode = "wb" if isinstance(content, (bytes, bytearray, memoryview)) else "w"
        with open(path, mode) as f:
            f.write(content)
            f.flush()
            os.fsync(f.fileno())

    def write_state_dict(self, state_dict, path, write_func=None):
        path = str(path)
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        if write_func:
            write_func(state_dict, path)

    def read(self, path, mode="r"):
        path = str(path)
        if not os.path.exists(path):
            return ""
        with open(path, mode) as f:
            return f.read()

    def read_state_dict(self, path, read_func):
        path = str(path)
        if not read_func or not os.path.exists(path):
            return {}
        return read_func(path)

    def safe_rmtree(self, dir):
        if os.path.exists(dir):
            shutil.rmtree(dir, ignore_errors=True)

    def safe_remove(self, path):
        try:
            os.remove(path)
        except FileNotFoundError:
            pass

    def safe_makedirs(self, dir):
        os.makedirs(dir, exist_ok=True)

    def safe_move(self, src_path, dst_path):
        if os.path.exists(src_path) and not os.path.exists(dst_path):
            shutil.move(src_path, dst_path)

    def commit(self, step, success):
        logger.info(f"checkpoint step {step} persisted: {success}")

    def exists(self, path: str):
        return os.path.exists(path)

    def listdir(self, path: str):
        return os.listdir(path)

    def get_class_meta(self):
        return ClassMeta(module_path=type(self).__module__, class_name=type(self).__name__)

    def write_bytes(self, addr, nbytes, path, offset=0, truncate=True, fsync=True, threads=8):
        path = str(path)
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        mode = (1 if truncate else 0) | (2 if fsync else 0) | _direct_bit()
        r = runtime().dw_write_file(path.encode(), ctypes.c_void_p(addr), int(nbytes), int(offset),
                                    int(threads), mode)
        if r != 0:
            raise OSError(f"write {path}: {last_error()}")

    def read_into(self, path, addr, nbytes, offset=0, threads=8):
        r = runtime().dw_read_file(str(path).encode(), ctypes.c_void_p(addr), int(nbytes), int(offset),
                                   int(threads))
        if r != 0:
            raise OSError(f"read {path}: {last_error()}")


class CheckpointDeletionStrategy(ABC):
    @abstractmethod
    def clean_up(self, step: int, delete_func: Callable):
        """Delete what should not be kept once ``step`` is committed."""


class KeepStepIntervalStrategy(CheckpointDeletionStrategy):
    """Keep only steps that are multiples of ``keep_interval``."""

    def __init__(self, keep_interval: int, checkpoint_dir: str, dir_format: str = "{}"):
        self._keep_interval = keep_interval
        self._checkpoint_dir = checkpoint_dir
        self._dir_format = dir_format  # step -> directory name (Megatron: "iter_{:07d}")

    def clean_up(self, step, delete_func):
        if self._keep_interval > 0 and step % self._keep_interval == 0:
            return
        target = os.path.join(self._checkpoint_dir, self._dir_format.format(step))
        try:
            delete_func(target)
        except Exception:
            logger.warning(f"cannot clean {target}")


class KeepLatestStepStrategy(CheckpointDeletionStrategy):
    """Keep the newest ``max_to_keep`` steps."""

    def __init__(self, max_to_keep: int, checkpoint_dir: str, dir_format: str = "{}"):
        self._max_to_keep = max(1, max_to_keep)
        self._checkpoint_dir = checkpoint_dir
        self._dir_format = dir_format
        self._steps: List[int] = []

    def clean_up(self, step, delete_func):
        self._steps.append(step)
        while len(self._steps) >= self._max_to_keep:
            old = self._steps.pop(0)
            target = os.path.join(self._checkpoint_dir, self._dir_format.format(old))
            try:
                delete_func(target)
            except Exception:
                logger.warning(f"cannot clean {target}")


class PosixStorageWithDeletion(PosixDiskStorage):
    """Applies a deletion strategy to the previously committed step."""

    def __init__(self, tracker_file: str, deletion_strategy: CheckpointDeletionStrategy):
        super().__init__()
        self._tracker_file = tracker_file
        self._deletion_strategy = deletion_strategy
        self._pre_step = 0

    def write(self, content, path):
        path = str(path)
        if path.endswith(self._tracker_file):
            prev = self.read(path)
            if prev and prev.strip().isdigit():
                self._pre_step = int(prev.strip())
        super().write(content, path)

    def commit(self, step, success):
        super().commit(step, success)
        if success and self._pre_step and self._pre_step != step:
            self._deletion_strategy.clean_up(self._pre_step, shutil.rmtree)

    def get_class_meta(self):
        return ClassMeta(module_path=type(self).__module__, class_name=type(self).__name__,
                         kwargs={"tracker_file": self._tracker_file,
                                 "deletion_strategy": self._deletion_strategy})


def get_checkpoint_storage(deletion_strategy: Optional[CheckpointDeletionStrategy] = None) -> CheckpointStorage:
    if deletion_strategy is not None:
        return PosixStorageWithDeletion(tracker_file=CheckpointConstant.TRACER_FILE_NAME,
                                        deletion_strategy=deletion_strategy)
    return PosixDiskStorage()
