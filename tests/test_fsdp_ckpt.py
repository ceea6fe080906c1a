"""FSDP flash checkpoint on CPU/gloo: memory snapshot + in-place restore,
DCP-compatible persistence (read back with torch's own FileSystemReader, also
at a different world size), storage fallback (parity: reference
``dlrover/trainer/tests/torch/fsdp_ckpt_test.py``)."""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))


def _train(model, opt, seed):
    g = torch.Generator().manual_seed(seed)
    model(torch.randn(4, 8, generator=g)).pow(2).sum().backward()
    opt.step()
    opt.zero_grad()


def _local(model):
    return {k: v.to_local().clone() for k, v in model.state_dict().items()}


def _fsdp_worker(rank, world, port, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from torch.distributed.fsdp import fully_shard

        from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
        from dlrover_wuqiong_amd.flash_checkpoint.fsdp import FsdpShardCheckpointer, wait_for_persist

        model = _model()
        for m in model:
            if isinstance(m, torch.nn.Linear):
                fully_shard(m)
        fully_shard(model)
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
        _train(model, opt, 1)
        ck = FsdpShardCheckpointer(root)
        proj = torch.arange(12.0).view(3, 4)  # saved through a non-contiguous view
        # one-time shm set-up ahead of the first save, with the same layout
        assert ck.prepare(model, opt, {"epoch": 7, "proj": proj.t()})
        assert ck.save_checkpoint(2, model, opt, {"epoch": 7, "proj": proj.t()}, storage_type=StorageType.MEMORY)
        assert ck.engine._planner.fast_hits >= 1  # the save reused prepare()'s DCP plan
        ck.wait_latest_checkpoint()
        want = _local(model)
        want_m = {k: v.to_local().clone() for k, v in opt.state_dict()["state"][0].items()
                  if torch.is_tensor(v) and hasattr(v, "to_local")}
        _train(model, opt, 2)
        _train(model, opt, 3)
        proj.zero_()
        extra = ck.load_checkpoint(model, opt, extra_sd={"epoch": 0, "proj": proj.t()})
        got = _local(model)
        ok = extra.get("epoch") == 7 and extra.get("step") == 2
        ok = ok and torch.equal(proj, torch.arange(12.0).view(3, 4))  # restored through the live view
        ok = ok and all(torch.equal(got[k], want[k]) for k in want)
        st = opt.state_dict()["state"][0]
        ok = ok and all(torch.equal(st[k].to_local(), v) for k, v in want_m.items())
        # training continues identically after the restore
        _train(model, opt, 4)
        # persist (DCP layout written by local rank 0's saver thread)
        assert ck.save_checkpoint(5, model, opt, {"epoch": 8}, storage_type=StorageType.DISK)
        want5 = _local(model)
        if rank == 0:
            ok = ok and wait_for_persist(root, 5, timeout=60)
        dist.barrier()
        # storage path: torch's own DCP reader into a fresh FSDP model
        import torch.distributed.checkpoint as dist_cp

        sd = {"model": model.state_dict()}
        for v in sd["model"].values():
            v.to_local().zero_()
        dist_cp.load(sd, storage_reader=dist_cp.FileSystemReader(os.path.join(root, "5")))
        ok = ok and all(torch.equal(v.to_local(), want5[k]) for k, v in sd["model"].items())
        # engine fallback to storage (memory skipped)
        for v in model.state_dict().values():
            v.to_local().zero_()
        sd2 = ck._state(model, opt, {"epoch": 0})
        step = ck.engine._load_from_storage_dcp(sd2)
        ok = ok and step == 5 and sd2["epoch"] == 8
        # same world size and sharding: the fast reader (O_DIRECT ranges of
        # the .distcp files straight into the live shards), not dist_cp.load
        ok = ok and ck.engine.last_restore_source == "storage"
        ok = ok and ck.engine.last_storage_load_stats.get("fast") is True
        got5 = _local(model)
        ok = ok and all(torch.equal(got5[k], want5[k]) for k in want5)
        ck.close()
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover - surfaced through the queue
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_fsdp_shard_checkpoint_two_ranks(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    root = str(tmp_path / "ck")
    ps = [ctx.Process(target=_fsdp_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)], res
    # reshard on read: a single process loads the 2-rank checkpoint as full tensors
    import torch.distributed.checkpoint as dist_cp

    ref = _model()
    sd = {"model": {k: torch.zeros_like(v) for k, v in ref.state_dict().items()}}
    dist_cp.load(sd, checkpoint_id=os.path.join(root, "5"), no_dist=True)
    assert all(v.abs().sum() > 0 for v in sd["model"].values())
    assert not os.path.exists(os.path.join(root, "5", ".dwamd_dcp_parts"))
