"""Megatron distributed-optimizer flash checkpoint at 4 gloo ranks with a
stand-in Megatron package and a fake DistributedOptimizer (each rank owns a
1/4 slice of the flattened parameters): per-rank ``rank_XXXXX/distrib_optim
.pt`` files holding only the local shard (no DP gather), in-place restore
from memory, parallel per-rank load from storage, iter_* deletion strategies.
Parity: reference dlrover/trainer/tests/torch/megatron_dist_ckpt_test.py
(behaviour), megatron_dist_ckpt.py:176-680."""

import os
import sys
import textwrap
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port

FAKE = {
    "megatron/__init__.py": "",
    "megatron/training/__init__.py": """
        import types
        ARGS = types.SimpleNamespace(save=None, load=None, use_distributed_optimizer=True, no_save_optim=False,
                                     no_save_rng=False, no_load_optim=False, no_load_rng=False, finetune=False,
                                     consumed_train_samples=0, consumed_valid_samples=0)
        def get_args():
            return ARGS
    """,
    "megatron/training/utils.py": """
        def print_rank_0(*a):
            pass
        def unwrap_model(m):
            return m
    """,
    "megatron/training/checkpointing.py": """
        import os, random
        import numpy as np
        import torch
        def get_checkpoint_name(path, iteration, release=False):
            d = "release" if release else f"iter_{iteration:07d}"
            return os.path.join(path, d, "mp_rank_00", "model_optim_rng.pt")
        def get_rng_state():
            return [{"random_rng_state": random.getstate(), "np_rng_state": np.random.get_state(),
                     "torch_rng_state": torch.get_rng_state(), "cuda_rng_state": None, "rng_tracker_states": {}}]
    """,
    "megatron/core/__init__.py": "from . import mpu",
    "megatron/core/mpu.py": """
        import torch.distributed as dist
        def get_data_parallel_rank():
            return dist.get_rank()
        def get_data_modulo_expert_parallel_rank():
            return dist.get_rank()
        def model_parallel_is_initialized():
            return True
        def get_tensor_model_parallel_rank():
            return 0
        def get_tensor_model_parallel_world_size():
            return 1
        def get_pipeline_model_parallel_rank():
            return 0
        def get_pipeline_model_parallel_world_size():
            return 1
    """,
}


class _Model(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.fc = torch.nn.Linear(16, 10)

    def state_dict_for_save_checkpoint(self):
        return self.state_dict()


class _FakeDistOpt:
    """Megatron DistributedOptimizer's shape: gbuf_ranges, the model-param ->
    (group, order) map and an inner Adam over this rank's fp32 main shard."""

    def __init__(self, model, rank, world):
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        per = (flat.numel() + world - 1) // world
        self.lo, self.hi = rank * per, min(flat.numel(), (rank + 1) * per)
        self.main = torch.nn.Parameter(flat[self.lo:self.hi].clone())
        self.optimizer = torch.optim.AdamW([self.main], lr=1e-2)
        key = model.fc.weight
        self.gbuf_ranges = [{torch.float32: [{"param_map": {key: (self.lo, self.hi)}}]}]
        self.model_param_group_index_map = {key: (0, 0)}

    def step(self, seed):
        g = torch.Generator().manual_seed(seed)
        self.main.grad = torch.randn(self.main.shape, generator=g)
        self.optimizer.step()

    def state_dict(self):
        return {"param_groups": self.optimizer.state_dict()["param_groups"]}

    def load_state_dict(self, sd):
        pass


def _worker(rank, world, port, root, fake_root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    sys.path.insert(0, fake_root)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import megatron.training as mt

        from dlrover_wuqiong_amd.flash_checkpoint import megatron_dist_ckpt as mdc
        from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType

        mt.ARGS.save = mt.ARGS.load = root
        model = _Model()
        opt = _FakeDistOpt(model, rank, world)
        opt.step(1)
        ok = True
        # ---- persisted save: every rank writes only its own shard
        assert mdc.save_checkpoint(10, model, opt, None, storage_type=StorageType.DISK)
        want10 = {"main": opt.main.detach().clone(), "m": opt.optimizer.state[opt.main]["exp_avg"].clone()}
        tracker = os.path.join(root, "latest_checkpointed_iteration.txt")
        deadline = time.time() + 60
        while time.time() < deadline and not (os.path.exists(tracker) and open(tracker).read().strip() == "10"):
            time.sleep(0.05)
        mine = os.path.join(root, "iter_0000010", f"rank_{rank:05d}", "distrib_optim.pt")
        ok = ok and os.path.exists(mine)
        shard = torch.load(mine, weights_only=True)
        ok = ok and shard[0][0][0]["param"].numel() == opt.hi - opt.lo  # local shard only: no DP gather
        ok = ok and os.path.exists(os.path.join(root, "iter_0000010", "mp_rank_00", "model_optim_rng.pt"))
        # ---- memory save, then an in-place restore of everything
        opt.step(2)
        with torch.no_grad():
            model.fc.weight.add_(1.0)
        assert mdc.save_checkpoint(20, model, opt, None, storage_type=StorageType.MEMORY)
        want20 = {"main": opt.main.detach().clone(), "m": opt.optimizer.state[opt.main]["exp_avg"].clone(),
                  "w": model.fc.weight.detach().clone()}
        opt.step(3)
        with torch.no_grad():
            model.fc.weight.zero_()
        it, _flops = mdc.load_checkpoint(model, opt, None)
        ok = ok and it == 20 and torch.equal(opt.main.detach(), want20["main"])
        ok = ok and torch.equal(opt.optimizer.state[opt.main]["exp_avg"], want20["m"])
        ok = ok and torch.equal(model.fc.weight.detach(), want20["w"])
        # ---- parallel per-rank load from storage (memory miss): own file only
        import megatron.training.checkpointing as mck  # noqa: F401

        m = mdc._mlm()
        msd, osd, _rel = mdc._load_from_storage(m, root, True)
        mdc.load_parameter_state_from_state_dict(opt, osd)
        ok = ok and msd["iteration"] == 10 and torch.equal(opt.main.detach(), want10["main"])
        ok = ok and torch.equal(opt.optimizer.state[opt.main]["exp_avg"], want10["m"])
        mdc.MegatronDistCheckpointer.reset_instances()
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_megatron_dist_optimizer_four_ranks(tmp_path):
    fake_root = tmp_path / "fake"
    for rel, src in FAKE.items():
        p = fake_root / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(textwrap.dedent(src))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    root = str(tmp_path / "ck")
    ps = [ctx.Process(target=_worker, args=(r, 4, port, root, str(fake_root), q)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == [(r, True) for r in range(4)], res


def test_iter_dir_deletion_strategies(tmp_path):
    from dlrover_wuqiong_amd.flash_checkpoint.megatron_dist_ckpt import KeepLatestStepStrategy, KeepStepIntervalStrategy

    removed = []
    s = KeepStepIntervalStrategy(100, str(tmp_path))
    s.clean_up(100, removed.append)
    s.clean_up(150, removed.append)
    assert removed == [os.path.join(str(tmp_path), "iter_0000150")]
    removed.clear()
    k = KeepLatestStepStrategy(2, str(tmp_path))
    for step in (10, 20, 30):
        k.clean_up(step, removed.append)
    assert removed and removed[0] == os.path.join(str(tmp_path), "iter_0000010")
