"""Flash checkpoint for DeepSpeed engines (ZeRO 0-3), DeepSpeed file layout.

``DeepSpeedEngine.save_checkpoint`` writes ``{dir}/{tag}/mp_rank_XX_model_states.pt``
and, with ZeRO, one ``zero_pp_rank_R_mp_rank_XX_optim_states.pt`` per rank,
all through ``torch.save``.  The checkpointer captures those writes
(``framework_io.py``), snapshots them into shared memory with the flash engine
and lets the agent persist them to the same paths, then commits DeepSpeed's
``latest`` tracker; ``load_checkpoint`` serves DeepSpeed's ``torch.load`` calls
from memory when every rank holds the same step.

Saving ranks: with ZeRO every rank owns an optimizer shard (local shards =
local world); without ZeRO only local rank 0 of each node saves (DeepSpeed's
``save_non_zero_checkpoint`` is enabled there so every node keeps a model copy
for its own restart).

Parity: reference ``flash_checkpoint/deepspeed.py`` (``AsyncCheckpointAgent``
:45-96, ``DeepSpeedCheckpointer`` :98-283) and ``deepspeed_engine.py``.
DeepSpeed itself is not importable in this image: the tests drive the
checkpointer with an engine object exposing the same methods
(``tests/test_framework_ckpt.py``).
"""

import os
from typing import Optional

import torch.distributed as dist

from ..common import env_utils
from ..common.constants import CheckpointConstant
from ..common.storage import get_checkpoint_storage
from .checkpointer import Checkpointer, StorageType
from .engine import FullCheckpointEngine
from .framework_io import TorchIOInterceptor, tag_to_step

DS_MODEL_SD_FILE_SUFFIX = "model_states.pt"
DS_OPTIM_SD_FILE_SUFFIX = "optim_states.pt"
DS_TRACER_FILE = "latest"
TAG_KEY = "__tag__"
ZERO_STAGE_WEIGHTS = 3


def _classify(path: str) -> Optional[str]:
    if path.endswith(DS_MODEL_SD_FILE_SUFFIX):
        return CheckpointConstant.MODEL_STATES_NAME
    if path.endswith(DS_OPTIM_SD_FILE_SUFFIX):
        return CheckpointConstant.OPTIM_STATES_NAME
    return os.path.basename(path)


class DeepSpeedCheckpointEngine(FullCheckpointEngine):
    def __init__(self, checkpoint_dir, storage=None, global_shard_num=1, zero_stage=0, comm_backend="",
                 save_timeout=CheckpointConstant.SAVE_TIMEOUT):
        self.zero_stage = zero_stage
        lw = max(1, env_utils.get_local_world_size())
        super().__init__(checkpoint_dir, storage, local_shard_num=min(lw, max(1, global_shard_num)),
                         global_shard_num=max(1, global_shard_num), comm_backend=comm_backend,
                         save_timeout=save_timeout, replicated=False)

    def get_saver_class(self):
        from ..elastic_agent.ckpt_saver import DeepSpeedCheckpointSaver

        return DeepSpeedCheckpointSaver

    def load(self, resume_path="", target=None):
        _step, sd = self.get_state_dict_from_memory(target=target)
        return sd or {}


class DeepSpeedCheckpointer(Checkpointer):
    """``engine``: a ``deepspeed.DeepSpeedEngine`` (or anything with its
    ``save_checkpoint`` / ``load_checkpoint`` / ``zero_optimization*`` API)."""

    def __init__(self, engine, checkpoint_dir, comm_backend="", deletion_strategy=None,
                 save_timeout=CheckpointConstant.SAVE_TIMEOUT, storage=None):
        self.engine = engine
        self.checkpoint_dir = checkpoint_dir
        global_shard_num = 1
        if engine.zero_optimization():
            group = getattr(getattr(engine, "optimizer", None), "dp_process_group", None)
            global_shard_num = dist.get_world_size(group) if dist.is_initialized() else 1
        zero_stage = engine.zero_optimization_stage()
        self.storage = storage or get_checkpoint_storage(deletion_strategy)
        self._async_save_engine = DeepSpeedCheckpointEngine(checkpoint_dir, storage=self.storage,
                                                            global_shard_num=global_shard_num,
                                                            zero_stage=zero_stage, comm_backend=comm_backend,
                                                            save_timeout=save_timeout)
        self.io = TorchIOInterceptor(_classify, self.storage)
        self._local_rank = env_utils.get_local_rank()
        self._ds_tracer_file = os.path.join(checkpoint_dir, DS_TRACER_FILE)
        self._dlrover_tracer_file = os.path.join(checkpoint_dir, CheckpointConstant.TRACER_FILE_NAME)
        if zero_stage < ZERO_STAGE_WEIGHTS and self._local_rank == 0:
            # every node keeps the (replicated) model states for its own restart
            engine.save_non_zero_checkpoint = True

    @property
    def flash_engine(self):
        return self._async_save_engine

    def save_checkpoint(self, save_dir, tag=None, client_state=None, save_latest=True,
                        storage_type=StorageType.DISK):
        tag = tag if tag is not None else f"global_step{self.engine.global_steps}"
        step = tag_to_step(tag)
        with self.io.capturing():
            self.engine.save_checkpoint(save_dir, tag, client_state or {}, save_latest)
        sd, paths = dict(self.io.state_dict), dict(self.io.paths)
        self.io.reset()
        paths[TAG_KEY] = str(tag)
        if storage_type == StorageType.MEMORY:
            ok = self._async_save_engine.save_to_memory(step, sd, paths)
            self._update_tracer_file(tag)
        elif storage_type == StorageType.DISK:
            self._update_tracer_file(tag)
            ok = self._async_save_engine.save_to_storage(step, sd, paths)
        else:
            raise ValueError(f"unsupported storage type {storage_type}")
        return ok

    def _update_tracer_file(self, tag):
        """DeepSpeed already rewrote ``latest`` and created ``{tag}/`` although
        nothing is on storage yet: undo both (the agent commits them)."""
        rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        if rank != 0:
            return
        self.storage.safe_rmtree(os.path.join(self.checkpoint_dir, str(tag)))
        content = self.storage.read(self._dlrover_tracer_file)
        if content:
            tags = self.storage.read(os.path.join(self.checkpoint_dir, "._dlrover_ds_tags", str(content).strip()))
            self.storage.write(tags or str(content), self._ds_tracer_file)
        else:
            self.storage.safe_remove(self._ds_tracer_file)

    def load_checkpoint(self, load_dir, tag=None, load_module_strict=True, load_optimizer_states=True,
                        load_lr_scheduler_states=True, load_module_only=False, custom_load_fn=None):
        sd = self._async_save_engine.load()
        kwargs = dict(load_module_strict=load_module_strict, load_optimizer_states=load_optimizer_states,
                      load_lr_scheduler_states=load_lr_scheduler_states, load_module_only=load_module_only)
        if custom_load_fn is not None:
            kwargs["custom_load_fn"] = custom_load_fn
        with self.io.serving(sd):
            return self.engine.load_checkpoint(load_dir, tag, **kwargs)

    def wait_latest_checkpoint(self):
        self._async_save_engine.wait_for_memory_save()

    def close(self):
        self._async_save_engine.close()
