"""Megatron-LM distributed-optimizer flash checkpoint: no data-parallel
gather on save, parallel per-rank load.

Megatron's own ``save_checkpoint`` with ``--use-distributed-optimizer``
gathers every DP rank's optimizer shard onto DP rank 0 (``get_parameter_state``
all-gathers into world-sized CPU buffers) before writing one
``distrib_optim.pt`` per model shard, and its load scatters them back.  Here
each rank keeps ITS OWN shard:

* save: ``get_parameter_state(opt)`` returns the live local shard tensors
  (fp32 main params + Adam moments per (bucket, group, order)) -- views, no
  copy, no collective.  The flash engine snapshots them to this rank's shm
  slice (``MegatronDistCheckpointEngine``: every rank is a shard) and the
  agent persists ``iter_XXXXXXX/rank_{rank:05d}/distrib_optim.pt`` next to
  Megatron's ``mp_rank_*/model_optim_rng.pt`` (written by DP rank 0 of each
  model shard);
* load: from shm when the step is in memory, else every rank reads only its
  own ``rank_XXXXX`` file (all ranks in parallel) and copies it into its
  shard (``load_parameter_state_from_state_dict``).

Model states are kept in memory on every DP rank (cheap next to the sharded
optimizer states) so an in-memory restore needs no broadcast; only DP rank 0
of a model shard persists them.

Parity: reference dlrover/trainer/torch/flash_checkpoint/megatron_dist_ckpt.py
(deletion strategies :78-147, save_checkpoint :176-295, checkpoint name
:298-311, get_parameter_state :314-358, load_checkpoint :372-587,
load_parameter_state_from_state_dict :650-680).  Megatron-LM is not importable
here: the save/load wrappers resolve its functions lazily and the tests drive
them with a stand-in package (parity unpinned against real Megatron).
"""

import os
import random
import types
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..common.constants import CheckpointConstant
from ..common.log import logger
from ..common.serialize import safe_torch_load
from ..common.storage import KeepLatestStepStrategy as _KeepLatest
from ..common.storage import KeepStepIntervalStrategy as _KeepInterval
from ..common.storage import get_checkpoint_storage
from .checkpointer import StorageType
from .megatron import (MEGATRON_TRACER_FILE, MegatronCheckpointEngine, MegatronDistCheckpointEngine,
                       get_dist_optimizer_checkpoint_name)

__all__ = ["KeepStepIntervalStrategy", "KeepLatestStepStrategy", "MegatronDistCheckpointer", "save_checkpoint",
           "load_checkpoint", "get_parameter_state", "get_chained_optimizer_parameter_state",
           "load_parameter_state_from_state_dict", "load_chained_optimizer_parameter_state",
           "get_dist_optimizer_checkpoint_name"]


class KeepStepIntervalStrategy(_KeepInterval):
    """Keep ``iter_XXXXXXX`` directories whose iteration is a multiple of
    ``keep_interval``; delete the others once a newer one is committed."""

    def __init__(self, keep_interval: int, checkpoint_dir: str):
        super().__init__(keep_interval, checkpoint_dir, dir_format="iter_{:07d}")


class KeepLatestStepStrategy(_KeepLatest):
    """Keep the newest ``max_to_keep`` ``iter_XXXXXXX`` directories."""

    def __init__(self, max_to_keep: int, checkpoint_dir: str):
        super().__init__(max_to_keep, checkpoint_dir, dir_format="iter_{:07d}")


class MegatronDistCheckpointer:
    """Per-save-dir singleton choosing the engine by optimizer kind."""

    _instances: Dict[str, "MegatronDistCheckpointer"] = {}

    def __init__(self, checkpoint_dir, storage=None, comm_backend="", use_distributed_optimizer=False,
                 save_timeout=CheckpointConstant.SAVE_TIMEOUT, replica_count=0):
        self.checkpoint_dir = checkpoint_dir
        self.storage = storage or get_checkpoint_storage()
        cls = MegatronDistCheckpointEngine if use_distributed_optimizer else MegatronCheckpointEngine
        self.engine = cls(checkpoint_dir, self.storage, comm_backend, save_timeout, replica_count)

    @classmethod
    def singleton_instance(cls, checkpoint_dir, **kwargs) -> "MegatronDistCheckpointer":
        inst = cls._instances.get(checkpoint_dir)
        if inst is None:
            inst = cls._instances[checkpoint_dir] = cls(checkpoint_dir, **kwargs)
        return inst

    @classmethod
    def reset_instances(cls):
        for inst in cls._instances.values():
            inst.engine.close()
        cls._instances = {}


# ------------------------------------------------------ optimizer shard state
def _param_slots(dist_optimizer):
    """Yield (bucket_idx, group_index, group_order, main_param) for every
    parameter range this rank's DistributedOptimizer owns."""
    for gbuf_range_maps in dist_optimizer.gbuf_ranges:
        if len(gbuf_range_maps) != 1:
            raise ValueError("one grad-buffer dtype per model chunk is supported")
        for _dtype, buckets in gbuf_range_maps.items():
            for bucket_idx, gbuf_range_map in enumerate(buckets):
                for model_param in gbuf_range_map["param_map"]:
                    gi, go = dist_optimizer.model_param_group_index_map[model_param]
                    yield bucket_idx, gi, go, dist_optimizer.optimizer.param_groups[gi]["params"][go]


def get_parameter_state(dist_optimizer) -> Dict:
    """{bucket: {group: {order: {"param": main_param, **adam_state}}}} of this
    rank's shard -- the live tensors (views): no copy, no DP gather."""
    state: Dict = {}
    for b, gi, go, main in _param_slots(dist_optimizer):
        st = dist_optimizer.optimizer.state[main]
        state.setdefault(b, {}).setdefault(gi, {})[go] = {"param": main, **st}
    return state


def get_chained_optimizer_parameter_state(chained_optimizer) -> List[Optional[Dict]]:
    return [get_parameter_state(o) if hasattr(o, "gbuf_ranges") else None
            for o in chained_optimizer.chained_optimizers]


def load_parameter_state_from_state_dict(dist_optimizer, state_dict: Dict):
    """Copy a rank's own shard state (from shm or its rank file) in place."""
    with torch.no_grad():
        for b, gi, go, main in _param_slots(dist_optimizer):
            saved = state_dict[b][gi][go]
            live = {"param": main, **dist_optimizer.optimizer.state[main]}
            for k, t in live.items():
                src = saved[k]
                if torch.is_tensor(t):
                    if t.data_ptr() != (src.data_ptr() if torch.is_tensor(src) else -1):
                        t.data.copy_(src)
                else:
                    dist_optimizer.optimizer.state[main][k] = src


def load_chained_optimizer_parameter_state(chained_optimizer, states):
    for i, o in enumerate(chained_optimizer.chained_optimizers):
        if hasattr(o, "gbuf_ranges") and states and states[i] is not None:
            load_parameter_state_from_state_dict(o, states[i])


def _is_chained(optimizer) -> bool:
    return hasattr(optimizer, "chained_optimizers")


# ------------------------------------------------------------ Megatron glue
def _mlm():
    """Megatron-LM functions used by the wrappers (new layout first)."""
    ns = types.SimpleNamespace()
    try:
        from megatron.training import get_args
        from megatron.training import checkpointing as ckpt
        try:
            from megatron.training.utils import print_rank_0, unwrap_model
        except ImportError:
            from megatron.training import print_rank_0
            from megatron.training.utils import unwrap_model
    except ImportError:
        try:
            from megatron import checkpointing as ckpt
            from megatron import get_args
            from megatron.utils import print_rank_0, unwrap_model
        except ImportError as e:
            raise ImportError("Megatron-LM is not importable") from e
    try:
        from megatron.core import mpu
    except ImportError:  # old Megatron-LM
        from megatron import mpu
    ns.get_args, ns.ckpt, ns.print_rank_0, ns.unwrap_model, ns.mpu = get_args, ckpt, print_rank_0, unwrap_model, mpu
    return ns


def _expert_dp_rank(mpu) -> int:
    if not (dist.is_available() and dist.is_initialized()):
        return 0
    for name in ("get_data_modulo_expert_parallel_rank", "get_expert_data_parallel_rank",
                 "get_data_parallel_rank"):
        f = getattr(mpu, name, None)
        if f is not None:
            try:
                return int(f())
            except Exception:
                continue
    return 0


def _model_state(m, args, model, optimizer, opt_param_scheduler, iteration, flops) -> Dict:
    sd = {"args": args, "checkpoint_version": 3.0, "iteration": iteration,
          "num_floating_point_operations_so_far": flops}
    if len(model) == 1:
        sd["model"] = model[0].state_dict_for_save_checkpoint()
    else:
        for i, chunk in enumerate(model):
            m.mpu.set_virtual_pipeline_model_parallel_rank(i)
            sd[f"model{i}"] = chunk.state_dict_for_save_checkpoint()
    if not getattr(args, "no_save_optim", False):
        if optimizer is not None:
            sd["optimizer"] = optimizer.state_dict()
        if opt_param_scheduler is not None:
            sd["opt_param_scheduler"] = opt_param_scheduler.state_dict()
    if not getattr(args, "no_save_rng", False) and hasattr(m.ckpt, "get_rng_state"):
        sd["rng_state"] = m.ckpt.get_rng_state()
    return sd


def save_checkpoint(iteration, model, optimizer, opt_param_scheduler, num_floating_point_operations_so_far=0,
                    storage_type=StorageType.DISK, comm_backend="", deletion_strategy=None,
                    save_timeout=CheckpointConstant.SAVE_TIMEOUT, storage=None):
    """Drop-in for Megatron's ``save_checkpoint`` with per-rank distributed
    optimizer shards (no gather).  ``storage_type=MEMORY``: shm only (the
    agent persists later / at a breakpoint); ``DISK``: shm then persisted
    asynchronously by the agent."""
    m = _mlm()
    args = m.get_args()
    storage = storage or get_checkpoint_storage(deletion_strategy)
    ck = MegatronDistCheckpointer.singleton_instance(
        args.save, storage=storage, comm_backend=comm_backend,
        use_distributed_optimizer=getattr(args, "use_distributed_optimizer", False), save_timeout=save_timeout)
    model = m.unwrap_model(model)
    if not isinstance(model, (list, tuple)):
        model = [model]
    sds, paths = {}, {}
    if getattr(args, "use_distributed_optimizer", False) and not getattr(args, "no_save_optim", False) \
            and optimizer is not None:
        sds[CheckpointConstant.OPTIM_STATES_NAME] = (get_chained_optimizer_parameter_state(optimizer)
                                                    if _is_chained(optimizer) else get_parameter_state(optimizer))
        paths[CheckpointConstant.OPTIM_STATES_NAME] = get_dist_optimizer_checkpoint_name(args.save, iteration)
    dp0 = _expert_dp_rank(m.mpu) == 0
    if dp0 or getattr(args, "use_distributed_optimizer", False):
        sds[CheckpointConstant.MODEL_STATES_NAME] = _model_state(m, args, model, optimizer, opt_param_scheduler,
                                                                 iteration, num_floating_point_operations_so_far)
        if dp0:  # only DP rank 0 of each model shard persists the model states
            paths[CheckpointConstant.MODEL_STATES_NAME] = m.ckpt.get_checkpoint_name(args.save, iteration)
    if storage_type == StorageType.MEMORY:
        ok = ck.engine.save_to_memory(iteration, sds, paths)
    else:
        ok = ck.engine.save_to_storage(iteration, sds, paths)
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
    return ok


def _load_from_memory(ck, target=None) -> Tuple[Dict, Dict, int]:
    """(model states, optimizer shard states, step) from shm.  With a
    ``target`` of the saved structure (the live tensors), the engine restores
    straight into them (H2D into the optimizer shards, no CPU copy);
    otherwise zero-copy CPU views."""
    step, sd = (0, None)
    if target is not None:
        try:
            step, sd = ck.engine.get_state_dict_from_memory(target=target)
        except Exception as e:  # structure changed: fall back to CPU views
            logger.info(f"in-place restore not possible ({e}); reading CPU views")
            step, sd = 0, None
    if not sd:
        step, sd = ck.engine.get_state_dict_from_memory()
    if not sd:
        return {}, {}, 0
    return sd.get(CheckpointConstant.MODEL_STATES_NAME, {}), sd.get(CheckpointConstant.OPTIM_STATES_NAME, {}), step


def _load_from_storage(m, load_dir: str, use_dist_opt: bool) -> Tuple[Optional[Dict], Dict, bool]:
    """This rank's files only (every rank reads in parallel, no scatter)."""
    tracker = os.path.join(load_dir, MEGATRON_TRACER_FILE)
    if not os.path.isfile(tracker):
        return None, {}, False
    content = open(tracker).read().strip()
    release = content == "release"
    iteration = 0 if release else int(content)
    name = m.ckpt.get_checkpoint_name(load_dir, iteration, release)
    if not os.path.exists(name) and hasattr(m.ckpt, "find_checkpoint_rank_0"):
        name = m.ckpt.find_checkpoint_rank_0(load_dir, iteration, release) or name
    msd = safe_torch_load(name) if os.path.exists(name) else None
    osd = {}
    if use_dist_opt:
        oname = get_dist_optimizer_checkpoint_name(load_dir, iteration, release)
        if os.path.exists(oname):
            osd = safe_torch_load(oname)
    return msd, osd, release


def load_checkpoint(model, optimizer, opt_param_scheduler, load_arg="load", strict=True, comm_backend="",
                    deletion_strategy=None, save_timeout=CheckpointConstant.SAVE_TIMEOUT, storage=None):
    """Drop-in for Megatron's ``load_checkpoint``: shm first, else this
    rank's own files.  Returns ``(iteration, num_floating_point_operations)``."""
    m = _mlm()
    args = m.get_args()
    load_dir = getattr(args, load_arg)
    use_dist_opt = getattr(args, "use_distributed_optimizer", False)
    storage = storage or get_checkpoint_storage(deletion_strategy)
    ck = MegatronDistCheckpointer.singleton_instance(args.save, storage=storage, comm_backend=comm_backend,
                                                     use_distributed_optimizer=use_dist_opt,
                                                     save_timeout=save_timeout)
    model = m.unwrap_model(model)
    if not isinstance(model, (list, tuple)):
        model = [model]
    target = None
    if use_dist_opt and optimizer is not None:
        # the live tensors in the layout save_checkpoint snapshots
        target = {}
        if _expert_dp_rank(m.mpu) == 0 or use_dist_opt:
            target[CheckpointConstant.MODEL_STATES_NAME] = _model_state(m, args, model, optimizer,
                                                                        opt_param_scheduler, 0, 0)
        target[CheckpointConstant.OPTIM_STATES_NAME] = (get_chained_optimizer_parameter_state(optimizer)
                                                       if _is_chained(optimizer) else get_parameter_state(optimizer))
    msd, osd, step = _load_from_memory(ck, target)
    release = False
    if not msd:
        msd, osd, release = _load_from_storage(m, load_dir, use_dist_opt)
    if msd is None:
        if getattr(args, "exit_on_missing_checkpoint", False):
            raise SystemExit("--exit-on-missing-checkpoint: no checkpoint")
        return 0, 0
    if hasattr(m.ckpt, "set_checkpoint_version"):
        m.ckpt.set_checkpoint_version(msd.get("checkpoint_version", 0))
    finetune = getattr(args, "finetune", False)
    iteration = 0 if (finetune or release) else msd.get("iteration", msd.get("total_iters", 0))
    flops = msd.get("num_floating_point_operations_so_far", 0)
    if "args" in msd and not finetune:
        ca = msd["args"]
        if hasattr(m.ckpt, "check_checkpoint_args"):
            m.ckpt.check_checkpoint_args(ca)
        args.consumed_train_samples = getattr(ca, "consumed_train_samples", 0)
        args.consumed_valid_samples = getattr(ca, "consumed_valid_samples", 0)
        try:
            from megatron.core.num_microbatches_calculator import update_num_microbatches
        except ImportError:
            update_num_microbatches = getattr(m.ckpt, "update_num_microbatches", None)
        if update_num_microbatches is not None:
            update_num_microbatches(consumed_samples=args.consumed_train_samples)
    if len(model) == 1:
        model[0].load_state_dict(msd["model"], strict=strict)
    else:
        for i, chunk in enumerate(model):
            m.mpu.set_virtual_pipeline_model_parallel_rank(i)
            chunk.load_state_dict(msd[f"model{i}"], strict=strict)
    if hasattr(m.ckpt, "fix_query_key_value_ordering") and hasattr(m.ckpt, "get_checkpoint_version"):
        m.ckpt.fix_query_key_value_ordering(model, m.ckpt.get_checkpoint_version())
    if not release and not finetune and not getattr(args, "no_load_optim", False):
        if optimizer is not None and "optimizer" in msd:
            optimizer.load_state_dict(msd["optimizer"])
        if use_dist_opt and optimizer is not None and osd:
            if _is_chained(optimizer):
                load_chained_optimizer_parameter_state(optimizer, osd)
            else:
                load_parameter_state_from_state_dict(optimizer, osd)
        if opt_param_scheduler is not None:
            key = "lr_scheduler" if "lr_scheduler" in msd else "opt_param_scheduler"
            if key in msd:
                opt_param_scheduler.load_state_dict(msd[key])
    if not release and not finetune and not getattr(args, "no_load_rng", False) and "rng_state" in msd:
        _set_rng(msd["rng_state"], args, m)
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
    src = f"memory (step {step})" if step else "storage"
    logger.info(f"megatron distributed-optimizer checkpoint of iteration {iteration} loaded from {src}")
    return iteration, flops


def _set_rng(rng_states, args, m):
    rs = rng_states
    if isinstance(rs, (list, tuple)):
        idx = m.mpu.get_data_parallel_rank() if getattr(args, "data_parallel_random_init", False) else 0
        rs = rs[idx]
    random.setstate(rs["random_rng_state"])
    np.random.set_state(rs["np_rng_state"])
    torch.set_rng_state(rs["torch_rng_state"])
    if torch.cuda.is_available() and rs.get("cuda_rng_state") is not None:
        torch.cuda.set_rng_state(rs["cuda_rng_state"])
    tracker = rs.get("rng_tracker_states")
    if tracker:
        try:
            from megatron.core import tensor_parallel

            tensor_parallel.get_cuda_rng_tracker().set_states(tracker)
        except ImportError:
            pass
