"""Flash checkpoint for Megatron-LM-layout checkpoints.

Two entry points:

* ``save_checkpoint`` / ``load_checkpoint`` -- drop-in wrappers of
  Megatron-LM's own ``megatron.training.checkpointing`` functions (used when
  Megatron-LM is importable): its ``torch.save`` calls are captured
  (``framework_io.py``), snapshotted into shared memory, and persisted by the
  agent to exactly the paths Megatron chose (``iter_XXXXXXX/mp_rank_TT[_PPP]
  /model_optim_rng.pt``, ``.../distrib_optim.pt``), so Megatron's loaders
  and converters keep working.
* ``MegatronCheckpointer.save_checkpoint(iteration, state_dict, ...)`` -- the
  same layout for this framework's own TP/PP models (no Megatron needed);
  ranks come from ``parallel.state``.

Saving ranks: the first ``min(local_world, tp*pp)`` local ranks of a node
(data-parallel replicas of a model shard skip the snapshot; Megatron's rank
order puts TP/PP innermost, DP outer).  With the distributed optimizer every
rank owns an optimizer shard (``distrib_optim.pt``) and every rank saves.

Parity: reference ``flash_checkpoint/megatron.py`` (``MegatronCheckpointer``
:54-135, ``save_checkpoint`` :138-213, ``load_checkpoint`` :216-247),
``megatron_engine.py`` (``MegatronCheckpointEngine`` :28-157,
``MegatronDistCheckpointEngine`` :160-280) and the agent-side
``MegatronCheckpointSaver`` (tracker ``latest_checkpointed_iteration.txt``).
"""

import inspect
import os
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch.distributed as dist

from ..common import env_utils
from ..common.constants import CheckpointConstant
from ..common.log import logger
from ..common.serialize import safe_torch_load
from ..common.storage import get_checkpoint_storage
from .checkpointer import StorageType
from .engine import FullCheckpointEngine
from .framework_io import TorchIOInterceptor

MODEL_SD_NAME = "model_optim_rng.pt"
DIST_OPTIM_SD_NAME = "distrib_optim.pt"
MEGATRON_TRACER_FILE = "latest_checkpointed_iteration.txt"


@dataclass
class ParallelRanks:
    tp_rank: int = 0
    tp_size: int = 1
    pp_rank: int = 0
    pp_size: int = 1
    dp_rank: int = 0
    ep_rank: int = 0
    ep_size: int = 1


def parallel_ranks() -> ParallelRanks:
    """Megatron's ``mpu`` if initialised, else this framework's groups."""
    if dist.is_available() and dist.is_initialized():
        try:
            try:
                from megatron.core import mpu
            except ImportError:
                from megatron import mpu  # old Megatron-LM
            if mpu.model_parallel_is_initialized():
                return ParallelRanks(mpu.get_tensor_model_parallel_rank(), mpu.get_tensor_model_parallel_world_size(),
                                     mpu.get_pipeline_model_parallel_rank(),
                                     mpu.get_pipeline_model_parallel_world_size(), mpu.get_data_parallel_rank())
        except ImportError:
            pass
    from ..parallel import state

    if state.model_parallel_is_initialized():
        return ParallelRanks(state.get_tensor_model_parallel_rank(), state.get_tensor_model_parallel_world_size(),
                             state.get_pipeline_model_parallel_rank(),
                             state.get_pipeline_model_parallel_world_size(), state.get_data_parallel_rank(),
                             state.get_expert_model_parallel_rank(), state.get_expert_model_parallel_world_size())
    return ParallelRanks()


def get_checkpoint_name(checkpoints_path: str, iteration: int, release: bool = False,
                        ranks: Optional[ParallelRanks] = None) -> str:
    """Megatron-LM's ``get_checkpoint_name`` layout."""
    r = ranks or parallel_ranks()
    directory = "release" if release else f"iter_{iteration:07d}"
    common = f"mp_rank_{r.tp_rank:02d}" if r.pp_size == 1 else f"mp_rank_{r.tp_rank:02d}_{r.pp_rank:03d}"
    if r.ep_size > 1:
        common += f"_{r.ep_rank:03d}"
    return os.path.join(checkpoints_path, directory, common, MODEL_SD_NAME)


def get_dist_optimizer_checkpoint_name(checkpoints_path: str, iteration: int, release: bool = False) -> str:
    directory = "release" if release else f"iter_{iteration:07d}"
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    return os.path.join(checkpoints_path, directory, f"rank_{rank:05d}", DIST_OPTIM_SD_NAME)


def _classify(path: str) -> Optional[str]:
    if path.endswith(MODEL_SD_NAME):
        return CheckpointConstant.MODEL_STATES_NAME
    if path.endswith(DIST_OPTIM_SD_NAME):
        return CheckpointConstant.OPTIM_STATES_NAME
    return None


class MegatronCheckpointEngine(FullCheckpointEngine):
    """One shard per (tp, pp) model partition; DP replicas do not save."""

    def __init__(self, checkpoint_dir, storage=None, comm_backend="", save_timeout=CheckpointConstant.SAVE_TIMEOUT,
                 replica_count=0, ranks: Optional[ParallelRanks] = None):
        self.ranks = ranks or parallel_ranks()
        gsn = self.ranks.tp_size * self.ranks.pp_size
        lw = max(1, env_utils.get_local_world_size())
        super().__init__(checkpoint_dir, storage, local_shard_num=min(lw, gsn), global_shard_num=gsn,
                         comm_backend=comm_backend, save_timeout=save_timeout, replica_count=replica_count,
                         replicated=False)

    def get_saving_ranks(self):
        world = dist.get_world_size() if dist.is_initialized() else 1
        lw = max(1, env_utils.get_local_world_size())
        return [i for i in range(world) if i % lw < self.local_shard_num]

    def get_saver_class(self):
        from ..elastic_agent.ckpt_saver import MegatronCheckpointSaver

        return MegatronCheckpointSaver

    def load(self, resume_path="", target=None):
        _step, sd = self.get_state_dict_from_memory(target=target)
        return sd or {}


class MegatronDistCheckpointEngine(MegatronCheckpointEngine):
    """Distributed optimizer: every rank owns a ``distrib_optim.pt`` shard."""

    def __init__(self, checkpoint_dir, storage=None, comm_backend="", save_timeout=CheckpointConstant.SAVE_TIMEOUT,
                 replica_count=0, ranks: Optional[ParallelRanks] = None):
        self.ranks = ranks or parallel_ranks()
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        lw = max(1, env_utils.get_local_world_size())
        FullCheckpointEngine.__init__(self, checkpoint_dir, storage, local_shard_num=min(lw, world),
                                      global_shard_num=world, comm_backend=comm_backend, save_timeout=save_timeout,
                                      replica_count=replica_count, replicated=False)


class MegatronCheckpointer:
    """Per-checkpoint-dir singleton (Megatron's save/load are free functions)."""

    _instances: Dict[str, "MegatronCheckpointer"] = {}

    def __init__(self, checkpoint_dir, storage=None, comm_backend="", save_timeout=CheckpointConstant.SAVE_TIMEOUT,
                 replica_count=0, use_distributed_optimizer=False, deletion_strategy=None):
        self.checkpoint_dir = checkpoint_dir
        self.storage = storage or get_checkpoint_storage(deletion_strategy)
        cls = MegatronDistCheckpointEngine if use_distributed_optimizer else MegatronCheckpointEngine
        self.engine = cls(checkpoint_dir, self.storage, comm_backend, save_timeout, replica_count)
        self.io = TorchIOInterceptor(_classify, self.storage)

    @classmethod
    def singleton_instance(cls, checkpoint_dir, **kwargs) -> "MegatronCheckpointer":
        inst = cls._instances.get(checkpoint_dir)
        if inst is None:
            inst = cls(checkpoint_dir, **kwargs)
            cls._instances[checkpoint_dir] = inst
        return inst

    @classmethod
    def reset_instances(cls):
        for inst in cls._instances.values():
            inst.engine.close()
        cls._instances = {}

    # -------------------------------------------------- reference-style API
    @property
    def state_dict(self):
        return self.io.state_dict

    @property
    def paths(self):
        return self.io.paths

    def save(self, state_dict, path):
        if _classify(str(path)) is None:
            raise ValueError(f"MegatronCheckpointer only captures {MODEL_SD_NAME} / {DIST_OPTIM_SD_NAME} paths")
        self.io.save(state_dict, path)

    def load(self, path, **kwargs):
        sd = self.engine.load()
        with self.io.serving(sd):
            return self.io.load(path, **kwargs)

    def update_tracer_file(self, iteration: int):
        """Megatron rewrote its tracker and created ``iter_*`` although a
        memory-only save wrote nothing: drop the empty directory and point
        the tracker back at the last *persisted* iteration."""
        self.storage.safe_rmtree(os.path.join(self.checkpoint_dir, f"iter_{iteration:07d}"))
        tracker = os.path.join(self.checkpoint_dir, MEGATRON_TRACER_FILE)
        content = self.storage.read(os.path.join(self.checkpoint_dir, CheckpointConstant.TRACER_FILE_NAME))
        if content:
            self.storage.write(content, tracker)
        else:
            self.storage.safe_remove(tracker)

    def _flush_captured(self, iteration, storage_type) -> bool:
        sd, paths = dict(self.io.state_dict), dict(self.io.paths)
        self.io.reset()
        if storage_type == StorageType.MEMORY:
            return self.engine.save_to_memory(iteration, sd, paths)
        if storage_type == StorageType.DISK:
            return self.engine.save_to_storage(iteration, sd, paths)
        raise ValueError(f"unsupported storage type {storage_type}")

    # ------------------------------------------------------- native API
    def save_checkpoint(self, iteration: int, state_dict: Dict, optim_state: Optional[Dict] = None,
                        storage_type=StorageType.DISK) -> bool:
        """Save this framework's TP/PP model state in Megatron layout."""
        r = self.engine.ranks
        sd = {}
        paths = {}
        if r.dp_rank == 0 or isinstance(self.engine, MegatronDistCheckpointEngine):
            sd[CheckpointConstant.MODEL_STATES_NAME] = dict(state_dict, iteration=iteration, checkpoint_version=3.0)
            paths[CheckpointConstant.MODEL_STATES_NAME] = get_checkpoint_name(self.checkpoint_dir, iteration,
                                                                             ranks=r)
        if optim_state is not None:
            sd[CheckpointConstant.OPTIM_STATES_NAME] = optim_state
            paths[CheckpointConstant.OPTIM_STATES_NAME] = get_dist_optimizer_checkpoint_name(self.checkpoint_dir,
                                                                                            iteration)
        self.io.state_dict, self.io.paths = sd, paths
        return self._flush_captured(iteration, storage_type)

    def load_checkpoint(self, iteration: Optional[int] = None, target=None) -> Tuple[int, Dict]:
        """(iteration, {category: state}) from memory, else from storage."""
        step, sd = self.engine.get_state_dict_from_memory(target=target)
        if sd and (iteration is None or step == iteration):
            return step, sd
        if iteration is None:
            content = self.storage.read(os.path.join(self.checkpoint_dir, MEGATRON_TRACER_FILE))
            if not content:
                return 0, {}
            iteration = int(str(content).strip())
        import torch

        out = {}
        path = get_checkpoint_name(self.checkpoint_dir, iteration, ranks=self.engine.ranks)
        if os.path.exists(path):
            out[CheckpointConstant.MODEL_STATES_NAME] = safe_torch_load(path)
        opath = get_dist_optimizer_checkpoint_name(self.checkpoint_dir, iteration)
        if os.path.exists(opath):
            out[CheckpointConstant.OPTIM_STATES_NAME] = safe_torch_load(opath)
        return iteration, out

    def wait_latest_checkpoint(self):
        self.engine.wait_for_memory_save()

    def close(self):
        self.engine.close()


def _megatron():
    try:
        from megatron.training import get_args
        from megatron.training.checkpointing import load_checkpoint as mload
        from megatron.training.checkpointing import save_checkpoint as msave
    except ImportError:
        try:
            from megatron import get_args
            from megatron.checkpointing import load_checkpoint as mload
            from megatron.checkpointing import save_checkpoint as msave
        except ImportError as e:
            raise ImportError("Megatron-LM is not importable; use MegatronCheckpointer.save_checkpoint "
                              "for this framework's own models") from e
    return get_args, msave, mload


def save_checkpoint(iteration, model, optimizer, opt_param_scheduler, num_floating_point_operations_so_far=0,
                    storage_type=StorageType.DISK, storage=None, comm_backend="",
                    save_timeout=CheckpointConstant.SAVE_TIMEOUT, replica_count=0):
    """Drop-in for Megatron-LM's ``save_checkpoint`` (flash: memory first)."""
    get_args, msave, _ = _megatron()
    args = get_args()
    ck = MegatronCheckpointer.singleton_instance(
        args.save, storage=storage, comm_backend=comm_backend, save_timeout=save_timeout,
        replica_count=replica_count, use_distributed_optimizer=getattr(args, "use_distributed_optimizer", False))
    params = inspect.signature(msave).parameters
    with ck.io.capturing():
        if "num_floating_point_operations_so_far" in params:
            msave(iteration, model, optimizer, opt_param_scheduler, num_floating_point_operations_so_far)
        else:
            msave(iteration, model, optimizer, opt_param_scheduler)
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    if rank == 0:
        # Megatron already bumped its tracker; the agent commits it once every
        # shard is on storage
        ck.update_tracer_file(iteration)
    ok = ck._flush_captured(iteration, storage_type)
    logger.info(f"megatron flash checkpoint of iteration {iteration} ({storage_type.name}): {ok}")
    return ok


def load_checkpoint(model, optimizer, opt_param_scheduler, load_arg="load", strict=True, storage=None,
                    comm_backend="", save_timeout=CheckpointConstant.SAVE_TIMEOUT, replica_count=0):
    """Drop-in for Megatron-LM's ``load_checkpoint``: memory first, then the
    files Megatron names."""
    get_args, _, mload = _megatron()
    args = get_args()
    ck = MegatronCheckpointer.singleton_instance(
        args.save, storage=storage, comm_backend=comm_backend, save_timeout=save_timeout,
        replica_count=replica_count, use_distributed_optimizer=getattr(args, "use_distributed_optimizer", False))
    sd = ck.engine.load()
    with ck.io.serving(sd):
        return mload(model, optimizer, opt_param_scheduler, load_arg, strict)
