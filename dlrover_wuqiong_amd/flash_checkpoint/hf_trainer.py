"""Flash checkpointing for the HuggingFace ``transformers.Trainer``.

``FlashCkptTrainer`` is a drop-in ``Trainer``: every checkpoint the trainer
would write synchronously (model weights, optimizer, scheduler, scaler, RNG
state, DeepSpeed shards) is captured, snapshotted into shared memory by the
flash engine in (sub)seconds, and persisted by the agent to exactly the
files HF would have written (``model.safetensors`` in safetensors format,
``optimizer.pt`` ...).  Small JSON files (``config.json``,
``trainer_state.json``) are still written directly.  ``dlrover_latest.txt``
in the run directory names the last *complete* checkpoint step; resuming
uses HF's normal ``resume_from_checkpoint`` on those files.

Parity: reference ``flash_checkpoint/hf_trainer.py`` (``HfFlashCheckpointer``
:59, ``HfDeepSpeedCheckpointer`` :89, ``HfDdpCheckpointer`` :116,
``FlashCkptTrainer`` :132-330).  Differences: transformers 5 saves weights
with safetensors, so the weights are captured in ``_save`` and the agent
writes safetensors; every rank's captured files are persisted on its own
node (no node-0-only saver), so per-rank RNG files survive multi-node jobs.
"""

import os
from typing import Optional

import torch
import torch.distributed as dist

from ..common import env_utils
from ..common.constants import CheckpointConstant
from ..common.log import logger
from ..common.storage import get_checkpoint_storage
from .engine import FullCheckpointEngine
from .framework_io import TorchIOInterceptor

try:
    from transformers import Trainer
except ImportError as e:  # pragma: no cover
    raise ImportError("FlashCkptTrainer needs transformers") from e

SAFE_WEIGHTS_NAME = "model.safetensors"


class HfCheckpointEngine(FullCheckpointEngine):
    """One shard per rank (what each rank captured); every node persists
    its own ranks' files."""

    def __init__(self, checkpoint_dir, storage=None, comm_backend="", save_timeout=CheckpointConstant.SAVE_TIMEOUT):
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        lw = max(1, min(env_utils.get_local_world_size(), world))
        super().__init__(checkpoint_dir, storage, local_shard_num=lw, global_shard_num=world,
                         comm_backend=comm_backend, save_timeout=save_timeout, replicated=False)

    def get_saver_class(self):
        from ..elastic_agent.ckpt_saver import CommonDirCheckpointSaver

        return CommonDirCheckpointSaver


def _dedup_shared(state_dict):
    """safetensors refuses tensors that share storage (tied embeddings):
    keep the first name; ``from_pretrained`` re-ties."""
    seen, out = set(), {}
    for k, v in state_dict.items():
        if not torch.is_tensor(v):
            continue
        key = (v.untyped_storage().data_ptr(), v.storage_offset(), tuple(v.shape))
        if key in seen:
            continue
        seen.add(key)
        out[k] = v.detach().contiguous()
    return out


class FlashCkptTrainer(Trainer):
    """``transformers.Trainer`` with flash checkpoints (DDP or DeepSpeed)."""

    _flash_engine = None
    _flash_io: Optional[TorchIOInterceptor] = None
    _capturing = False

    def _get_flash(self, run_dir):
        if self._flash_engine is None:
            storage = get_checkpoint_storage()
            if getattr(self, "is_deepspeed_enabled", False):
                from .deepspeed import DeepSpeedCheckpointEngine

                eng = self.model_wrapped
                shards = dist.get_world_size(eng.optimizer.dp_process_group) if eng.zero_optimization() else 1
                self._flash_engine = DeepSpeedCheckpointEngine(run_dir, storage=storage, global_shard_num=shards,
                                                               zero_stage=eng.zero_optimization_stage())
            elif getattr(self, "is_fsdp_enabled", False):
                raise ValueError("FlashCkptTrainer supports DDP and DeepSpeed; use FsdpShardCheckpointer for FSDP")
            else:
                self._flash_engine = HfCheckpointEngine(run_dir, storage=storage)
            self._flash_io = TorchIOInterceptor(os.path.basename, storage)
        return self._flash_engine

    def _save_checkpoint(self, model, trial, *args, **kwargs):
        run_dir = self._get_output_dir(trial=trial)
        engine = self._get_flash(run_dir)
        self._capturing = True
        try:
            with self._flash_io.capturing():
                super()._save_checkpoint(model, trial, *args, **kwargs)
        finally:
            self._capturing = False
        sd, paths = dict(self._flash_io.state_dict), dict(self._flash_io.paths)
        self._flash_io.reset()
        ok = engine.save_to_storage(self.state.global_step, sd, paths)
        if not ok:
            logger.info(f"flash checkpoint of step {self.state.global_step} skipped: the previous one is "
                        "still being persisted")

    def _save(self, output_dir: Optional[str] = None, state_dict=None):
        if not self._capturing:
            return super()._save(output_dir, state_dict)
        output_dir = output_dir if output_dir is not None else self.args.output_dir
        os.makedirs(output_dir, exist_ok=True)
        model = self.accelerator.unwrap_model(self.model) if hasattr(self, "accelerator") else self.model
        if state_dict is None:
            state_dict = model.state_dict()
        self._flash_io.save(_dedup_shared(state_dict), os.path.join(output_dir, SAFE_WEIGHTS_NAME))
        cfg = getattr(model, "config", None)
        if cfg is not None and hasattr(cfg, "save_pretrained"):
            cfg.save_pretrained(output_dir)
        gen = getattr(model, "generation_config", None)
        if gen is not None and hasattr(gen, "save_pretrained"):
            try:
                gen.save_pretrained(output_dir)
            except Exception:  # generation config is optional
                pass
        if self.processing_class is not None:
            self.processing_class.save_pretrained(output_dir)
        torch.save(self.args, os.path.join(output_dir, "training_args.bin"))

    def wait_latest_checkpoint(self):
        if self._flash_engine is not None:
            self._flash_engine.wait_for_memory_save()
