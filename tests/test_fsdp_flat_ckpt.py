"""ATorch-style flat FSDP checkpoints (atorch/fsdp_flat_ckpt.py): 2 gloo
ranks flash-save FSDP2 shards + AdamW state; the agent-side saver writes
per-rank safetensors + JSON metadata; in-place memory restore; the files
load (resharded) into an unsharded model + fresh optimizer in one process
and reproduce the next training step exactly.  Parity: reference
atorch/tests/common_tests/fsdp_save_util_test.py (behaviour)."""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 30), torch.nn.ReLU(), torch.nn.Linear(30, 5))


def _batch(seed):
    return torch.randn(6, 8, generator=torch.Generator().manual_seed(seed))


def _worker(rank, world, port, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from torch.distributed.fsdp import fully_shard

        from dlrover_wuqiong_amd.atorch import fsdp_flat_ckpt as ffc
        from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType

        model = _model()
        for m in model:
            if isinstance(m, torch.nn.Linear):
                fully_shard(m)
        fully_shard(model)
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
        for s in range(2):
            model(_batch(s)).pow(2).sum().backward()
            opt.step()
            opt.zero_grad()
        path = os.path.join(root, "step-3")
        assert ffc.save_checkpoint(3, model, opt, path, storage_type=StorageType.DISK)
        ok = True
        if rank == 0:
            ok = ffc.wait_for_persist(root, 3, timeout=60)
        dist.barrier()
        ok = ok and os.path.exists(os.path.join(path, f"flat_param.{rank:05d}-00002"))
        full = {k: v.full_tensor().clone() for k, v in model.state_dict().items()}
        # next step's reference result (what a resharded restore must reproduce)
        model(_batch(9)).pow(2).sum().backward()
        opt.step()
        opt.zero_grad()
        after = {k: v.full_tensor().clone() for k, v in model.state_dict().items()}
        step = ffc.load_checkpoint(model, opt, path)  # in-place from shm
        ok = ok and step == 3 and all(torch.equal(v.full_tensor(), full[k]) for k, v in model.state_dict().items())
        if rank == 0:
            torch.save({"full": full, "after": after}, os.path.join(root, "ref.pt"))
        ffc.close_engines()
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_flat_ckpt_two_ranks_then_reshard_to_one(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == [(0, True), (1, True)], res

    from safetensors.torch import load_file

    from dlrover_wuqiong_amd.atorch.fsdp_flat_ckpt import ShardTensorUtil

    path = str(tmp_path / "step-3")
    assert open(tmp_path / "latest_checkpointed_iteration.txt").read().strip() == "3"
    shard0 = load_file(os.path.join(path, "flat_param.00000-00002"))  # plain safetensors
    assert shard0["0.weight"].shape == (15, 8)  # dim-0 shard of a [30, 8] weight
    ref = torch.load(tmp_path / "ref.pt", weights_only=True)
    util = ShardTensorUtil(path)
    assert torch.equal(util.load_tensor_by_name("0.weight"), ref["full"]["0.weight"])
    model = _model()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    util.load_into_model(model)
    util.load_optimizer(model, opt)
    for k, v in model.state_dict().items():
        assert torch.equal(v, ref["full"][k]), k
    model(_batch(9)).pow(2).sum().backward()
    opt.step()
    for k, v in model.state_dict().items():
        torch.testing.assert_close(v, ref["after"][k], rtol=1e-5, atol=1e-6)
