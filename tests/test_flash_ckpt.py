"""Flash checkpoint on CPU (gloo): layout, shm round trip, split (replicated)
save across ranks, persistence format, deletion strategies."""

import os
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def test_layout_coalesces_flat_views():
    from dlrover_wuqiong_amd.flash_checkpoint.layout import plan_layout

    flat = torch.arange(1000, dtype=torch.float32)
    sd = {"a": flat[0:100].view(10, 10), "b": flat[100:300], "c": {"d": flat[300:1000]}, "n": 3,
          "other": torch.ones(5)}
    layout, _ = plan_layout(sd)
    assert len(layout.extents) == 2  # one per storage
    assert layout.meta_tree["n"] == 3
    assert layout.meta_tree["c"]["d"].offset - layout.meta_tree["a"].offset == 300 * 4


def test_single_process_memory_roundtrip(tmp_path):
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer

    m = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 8))
    opt = torch.optim.AdamW(m.parameters())
    m(torch.randn(2, 32)).sum().backward()
    opt.step()
    ck = DdpCheckpointer(str(tmp_path / "ck"))
    sd = {"model": m.state_dict(), "optimizer": opt.state_dict(), "epoch": 3, "list": [1, torch.ones(2)]}
    assert ck.save_checkpoint(10, sd, storage_type=StorageType.MEMORY)
    out = ck.load_checkpoint()
    assert out["epoch"] == 3
    assert torch.equal(out["model"]["0.weight"], m[0].weight.detach())
    assert torch.equal(out["optimizer"]["state"][0]["exp_avg"], opt.state[m[0].weight]["exp_avg"])
    assert torch.equal(out["list"][1], torch.ones(2))
    # a new state of different size re-creates the segment
    sd2 = {"model": torch.nn.Linear(3, 3).state_dict()}
    assert ck.save_checkpoint(11, sd2, storage_type=StorageType.MEMORY)
    out2 = ck.load_checkpoint()
    assert set(out2["model"].keys()) == {"weight", "bias"}
    ck.close()


def test_prepare_sets_up_shm_before_first_save(tmp_path):
    """Checkpointer.prepare creates the segment and pins / prefaults the
    slots in the background; the first save then reuses it (no re-create)."""
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer

    m = torch.nn.Linear(64, 64)
    ck = DdpCheckpointer(str(tmp_path / "ck"))
    sd = {"model": m.state_dict(), "step": 1}
    assert ck.prepare(sd)
    eng = ck.engine
    assert eng._shm_prep is not None
    eng._shm_prep.result(timeout=60)
    ino, size = eng._shm_handler.shared_memory.ino, eng._shm_handler.payload_size
    assert size > 64 * 64 * 4
    assert ck.save_checkpoint(2, {"model": m.state_dict(), "step": 2}, storage_type=StorageType.MEMORY)
    assert eng._shm_handler.shared_memory.ino == ino and eng._shm_handler.payload_size == size
    assert ck.load_checkpoint()["step"] == 2
    ck.close()


def test_double_buffer_survives_torn_save(tmp_path):
    """A process dying mid-snapshot must leave the previous checkpoint intact."""
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer
    from dlrover_wuqiong_amd.flash_checkpoint.shm_handler import CheckpointConfig

    ck = DdpCheckpointer(str(tmp_path / "ck"))
    h = ck.engine._shm_handler
    for step in (4, 8):
        assert ck.save_checkpoint(step, {"w": torch.full((1000,), float(step))}, storage_type=StorageType.MEMORY)
    assert h.complete_steps() == {4: 0, 8: 1}
    # torn save of step 12: the writer invalidated its slot and died
    slot = h.write_slot()
    assert slot == 0
    h.set_slice_step(slot, 0, 0)
    h.set_metadata(slot, h.get_meta(1)["tree"], CheckpointConfig(step=12))
    h.payload_view(slot)[:16] = b"\xff" * 16
    assert h.complete_steps() == {8: 1}
    ck.close()
    # a restarted process restores step 8 and its first save goes to the other slot
    ck2 = DdpCheckpointer(str(tmp_path / "ck"))
    out = ck2.load_checkpoint()
    assert torch.equal(out["w"], torch.full((1000,), 8.0))
    assert ck2.save_checkpoint(16, {"w": torch.full((1000,), 16.0)}, storage_type=StorageType.MEMORY)
    assert ck2.engine._shm_handler.complete_steps() == {16: 0, 8: 1}
    ck2.close()


def test_slot_fallback_while_agent_persists(tmp_path):
    from dlrover_wuqiong_amd.common.multi_process import SharedLock
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer
    from dlrover_wuqiong_amd.flash_checkpoint.shm_handler import slot_lock_name

    ck = DdpCheckpointer(str(tmp_path / "ck"))
    h = ck.engine._shm_handler

    def save(step):
        return ck.save_checkpoint(step, {"w": torch.full((1000,), float(step))}, storage_type=StorageType.MEMORY)

    assert save(4) and save(8)
    assert h.complete_steps() == {4: 0, 8: 1}
    agent_lock = SharedLock(slot_lock_name(0, 0), create=True)
    assert agent_lock.acquire(blocking=False)  # the agent persists slot 0 (step 4)
    assert save(12)  # slot 0 busy -> slot 1 (slot 0 stays an intact checkpoint)
    assert h.complete_steps() == {4: 0, 12: 1}
    assert save(16)
    assert h.complete_steps() == {4: 0, 16: 1}
    agent_lock.release()
    assert save(20)
    assert h.complete_steps() == {20: 0, 16: 1}
    ck.close()


def test_save_to_storage_and_reload(tmp_path):
    from dlrover_wuqiong_amd.common.storage import KeepLatestStepStrategy
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer

    d = tmp_path / "ck"
    ck = DdpCheckpointer(str(d), deletion_strategy=KeepLatestStepStrategy(2, str(d)))
    for step in (1, 2, 3):
        sd = {"w": torch.full((100,), float(step))}
        assert ck.save_checkpoint(step, sd, storage_type=StorageType.DISK)
        deadline = time.time() + 30
        while time.time() < deadline:
            if (d / "dlrover_latest.txt").exists() and (d / "dlrover_latest.txt").read_text() == str(step):
                break
            time.sleep(0.05)
    assert (d / "dlrover_latest.txt").read_text() == "3"
    x = torch.load(d / "3" / "rank_0.pt", weights_only=True)
    assert torch.equal(x["w"], torch.full((100,), 3.0))
    # strategy keeps the newest 2 -> step 1 removed
    assert not (d / "1").exists()
    # fresh checkpointer with empty memory loads from storage
    ck.close()
    from dlrover_wuqiong_amd.flash_checkpoint.shm_handler import SharedMemoryHandler

    SharedMemoryHandler(0).unlink()
    ck2 = DdpCheckpointer(str(d))
    out = ck2.load_checkpoint()
    assert torch.equal(out["w"], torch.full((100,), 3.0))
    ck2.close()


def test_storage_restore_into_live_tensors(tmp_path):
    """Memory gone (node replaced): the persisted archive streams straight
    into the live tensors (O_DIRECT reads where the file system allows) and
    equals what torch.load returns."""
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer
    from dlrover_wuqiong_amd.flash_checkpoint.shm_handler import SharedMemoryHandler
    from dlrover_wuqiong_amd.flash_checkpoint.storage_loader import drop_file_cache

    d = tmp_path / "ck"
    flat = torch.randn(1 << 21)
    sd = {"model": {"w": flat[: 1 << 20].view(1024, 1024), "b": flat[1 << 20:]},
          "optimizer": {"state": {0: {"exp_avg": torch.randn(300, dtype=torch.bfloat16)}},
                        "param_groups": [{"lr": 0.5, "params": [0]}]},
          "t": torch.randn(6, 4).t(), "step": 9}
    ck = DdpCheckpointer(str(d))
    assert ck.save_checkpoint(9, sd, storage_type=StorageType.DISK)
    deadline = time.time() + 30
    while time.time() < deadline and not ((d / "dlrover_latest.txt").exists()
                                          and (d / "dlrover_latest.txt").read_text() == "9"):
        time.sleep(0.05)
    ck.close()
    SharedMemoryHandler(0).unlink()
    drop_file_cache(str(d / "9" / "rank_0.pt"))
    target = {"model": {"w": torch.zeros(1024, 1024), "b": torch.zeros(1 << 20)},
              "optimizer": {"state": {0: {"exp_avg": torch.zeros(300, dtype=torch.bfloat16)}},
                            "param_groups": [{"lr": 0.0, "params": [0]}]},
              "t": torch.zeros(4, 6), "step": 0}
    ck2 = DdpCheckpointer(str(d))
    out = ck2.load_checkpoint(target=target)
    assert ck2.engine.last_restore_source == "storage"
    assert out["model"]["w"] is target["model"]["w"]  # restored in place
    assert torch.equal(target["model"]["w"], sd["model"]["w"]) and torch.equal(target["model"]["b"], sd["model"]["b"])
    assert torch.equal(target["optimizer"]["state"][0]["exp_avg"], sd["optimizer"]["state"][0]["exp_avg"])
    assert torch.equal(target["t"], sd["t"]) and out["step"] == 9
    assert out["optimizer"]["param_groups"] == [{"lr": 0.5, "params": [0]}]
    assert ck2.engine.last_storage_load_stats["bytes_read"] >= flat.numel() * 4
    ck2.close()


def _split_worker(rank, world, port, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
        from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer

        torch.manual_seed(0)  # replicated state on every rank
        flat = torch.randn(3 << 20)
        sd = {"a": flat[: 1 << 20], "b": flat[1 << 20:], "meta": {"k": "v"}}
        ck = DdpCheckpointer(root)
        assert ck.engine._num_slices == world
        assert ck.save_checkpoint(4, sd, storage_type=StorageType.MEMORY)
        dist.barrier()
        h = ck.engine._shm_handler
        assert h.complete_step() == 4, h.complete_steps()
        out = ck.load_checkpoint()
        ok = torch.equal(out["a"], sd["a"]) and torch.equal(out["b"], sd["b"]) and out["meta"] == {"k": "v"}
        # persist through the saver of local rank 0
        assert ck.save_checkpoint(5, sd, storage_type=StorageType.DISK)
        dist.barrier()
        if rank == 0:
            deadline = time.time() + 60
            f = os.path.join(root, "dlrover_latest.txt")
            while time.time() < deadline and not os.path.exists(f):
                time.sleep(0.05)
            x = torch.load(os.path.join(root, "5", "rank_0.pt"), weights_only=False)
            ok = ok and torch.equal(x["b"], sd["b"])
        dist.barrier()
        ck.close()
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_replicated_split_save_two_ranks(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_split_worker, args=(r, 2, port, str(tmp_path / "ck"), q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


def test_overlapped_snapshot_fence_runs_before_any_optimizer_step():
    """copier.py's global optimizer step pre-hook fences pending snapshots
    (the GPU data path is covered by test_flash_ckpt_gpu.py)."""
    from dlrover_wuqiong_amd.flash_checkpoint import copier

    copier._install_fence_hook()
    copier._install_fence_hook()  # idempotent

    class _Pending:
        fenced = 0

        def fence(self):
            _Pending.fenced += 1

    p = _Pending()
    copier._FENCED.add(p)
    w = torch.nn.Parameter(torch.ones(3))
    opt = torch.optim.SGD([w], lr=0.1)
    w.sum().backward()
    opt.step()
    assert _Pending.fenced == 1 and len(copier._FENCED) == 0
    opt.step()
    assert _Pending.fenced == 1


def test_staging_ring_shape_follows_hbm_budget():
    """The staging ring grows from K x C to the HBM budget (never past the
    slice): explicit DWAMD_RING_HBM_GB, or the free HBM in auto mode."""
    from dlrover_wuqiong_amd.flash_checkpoint.copier import GpuCopier

    c = GpuCopier.__new__(GpuCopier)  # sizing logic only: no device needed
    c.ring_slots, c.ring_chunk, c.ring_hbm, c._ring_auto = 4, 1 << 30, 0, 0
    c.staging_mode = "ring"
    assert c._ring_shape(100 << 30) == (4, 1 << 30)  # forced ring: K x C
    c.ring_hbm = 64 << 30
    assert c._ring_shape(100 << 30) == (64, 1 << 30)
    assert c._ring_shape(10 << 30) == (10, 1 << 30)  # never beyond the slice
    c.ring_hbm, c.staging_mode, c._ring_auto = 0, "auto", 40 << 30
    assert c._ring_shape(100 << 30) == (40, 1 << 30)  # auto: the free HBM
    assert c._ring_shape(1 << 20)[0] == 4  # a tiny slice keeps the minimal ring


def test_shard_engine_load_falls_back_to_resume_path(tmp_path):
    """ShardCheckpointEngine with nothing in memory reads this rank's
    persisted shard from ``resume_path`` (it used to return {} silently)."""
    from dlrover_wuqiong_amd.flash_checkpoint.engine import ShardCheckpointEngine
    from dlrover_wuqiong_amd.flash_checkpoint.shm_handler import SharedMemoryHandler

    SharedMemoryHandler(0).unlink()
    p = tmp_path / "shard_0.pt"
    ref = {"w": torch.randn(257, 3), "step": 4}
    torch.save(ref, p)
    eng = ShardCheckpointEngine(str(tmp_path / "ck"))
    try:
        assert eng.load() == {}
        out = eng.load(resume_path=str(p))
        assert torch.equal(out["w"], ref["w"]) and out["step"] == 4
        tgt = {"w": torch.zeros(257, 3), "step": 0}
        out = eng.load(resume_path=str(p), target=tgt)
        assert torch.equal(tgt["w"], ref["w"])
    finally:
        eng.close()
