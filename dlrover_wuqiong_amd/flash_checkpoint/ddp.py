"""Flash checkpointer for DDP / replicated models.

Parity: reference ``dlrover/trainer/torch/flash_checkpoint/ddp.py:25-117``
(same constructor arguments and ``save_checkpoint``/``load_checkpoint``
semantics; the persisted file ``{dir}/{step}/rank_{rank}.pt`` is a plain
``torch.save`` of the state dict, loadable with ``torch.load``).

Extension: ``load_checkpoint(target=...)`` restores in place into live GPU
tensors (the fast path used for recovery: sliced H2D + xGMI all-gather).
"""

import os

import torch.distributed as dist

from ..common.constants import CheckpointConstant
from ..common.storage import get_checkpoint_storage
from .checkpointer import Checkpointer, StorageType
from .engine import FullCheckpointEngine


class DdpCheckpointer(Checkpointer):
    def __init__(self, checkpoint_dir: str, local_shard_num=1, global_shard_num=1, comm_backend="",
                 deletion_strategy=None, save_timeout=CheckpointConstant.SAVE_TIMEOUT, replica_count=0,
                 storage=None):
        self.checkpoint_dir = checkpoint_dir
        self._rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.storage = storage or get_checkpoint_storage(deletion_strategy)
        self._engine = FullCheckpointEngine(checkpoint_dir=checkpoint_dir, storage=self.storage,
                                            local_shard_num=local_shard_num, global_shard_num=global_shard_num,
                                            comm_backend=comm_backend, save_timeout=save_timeout,
                                            replica_count=replica_count)
        self._engine.defer_optimizer_restore = True

    @property
    def engine(self):
        return self._engine

    def save_checkpoint(self, step, state_dict, path="", storage_type=StorageType.DISK):
        if not path:
            path = os.path.join(self.checkpoint_dir, f"{step}/rank_{self._rank}.pt")
        sd = {CheckpointConstant.MODEL_STATES_NAME: state_dict}
        paths = {CheckpointConstant.MODEL_STATES_NAME: path}
        if storage_type == StorageType.MEMORY:
            return self._engine.save_to_memory(step, sd, paths)
        if storage_type == StorageType.DISK:
            return self._engine.save_to_storage(step, sd, paths)
        raise ValueError(f"unsupported storage type {storage_type}")

    def prepare(self, state_dict) -> bool:
        """Set up the shm slots for ``state_dict`` in the background (see
        ``CheckpointEngine.prepare_memory``), e.g. right after the first
        optimizer step, so the first memory save flushes at full speed."""
        return self._engine.prepare_memory({CheckpointConstant.MODEL_STATES_NAME: state_dict})

    def load_checkpoint(self, resume_path="", target=None):
        """Returns the state dict (from memory if possible, else storage).

        ``target``: optional state dict of live tensors with the saved
        structure; restored in place on the GPU fast path and returned.
        Restored from host memory, the tensors under an ``optim*`` key may
        still be landing when this returns (``deferred_restore.py``): the
        next ``optimizer.step()`` waits for them on the device; any other
        reader of that state first calls
        ``dlrover_wuqiong_amd.flash_checkpoint.deferred_restore.wait_all()``.
        """
        tgt = {CheckpointConstant.MODEL_STATES_NAME: target} if target is not None else None
        return self._engine.load(resume_path, target=tgt)

    def wait_latest_checkpoint(self, timeout=1800):
        """Block until the latest memory snapshot has landed in shm."""
        self._engine.wait_for_memory_save()

    def close(self):
        self._engine.close()
