"""Cross-node in-memory replicas (4 gloo ranks = 4 single-GPU "nodes",
replica_count=2 -> backup pairs {0,1}, {2,3}): backups ship off the save
path in raw chunks, a node whose shm is wiped (node replacement) restores its
own shard from its peer's replica (parity: reference
dlrover/trainer/tests/torch/checkpoint_replica_test.py)."""

import glob
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def _worker(rank, world, port, root, prefix, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", LOCAL_WORLD_SIZE="1", NODE_RANK=str(rank),
                      DWAMD_SHM_PREFIX=f"{prefix}n{rank}")  # one shm namespace per simulated node
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
        from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer

        ck = DdpCheckpointer(os.path.join(root, "ck"), replica_count=2)
        rm = ck.engine._replica_manager
        ok = rm.has_replica() and sorted(rm.backup_ranks) == ([0, 1] if rank < 2 else [2, 3])
        # rank-specific state so a restore from the wrong shard would show
        state = {"w": torch.arange(3_000_000, dtype=torch.float32) + 1000 * rank, "step": 5}
        ck.save_checkpoint(5, state, storage_type=StorageType.MEMORY)
        ck.wait_latest_checkpoint()
        rm.wait()
        ok = ok and rm.last_backup[0] == 5
        dist.barrier()
        ck.close()
        if rank == 1:  # node 1 replaced: its shm (own checkpoint + peer replicas) is gone
            gone = glob.glob(f"/dev/shm/dwamd_{prefix}n1*")
            ok = ok and any("checkpoint_shm" in f for f in gone) and any("replica_0" in f for f in gone)
            for f in gone:
                os.remove(f)
        dist.barrier()
        ck2 = DdpCheckpointer(os.path.join(root, "ck"), replica_count=2)
        target = {"w": torch.zeros(3_000_000), "step": 0}
        step, sd = ck2.engine.get_state_dict_from_memory()
        ok = ok and step == 5 and torch.equal(sd["model_states"]["w"], torch.arange(3_000_000, dtype=torch.float32)
                                                + 1000 * rank)
        del target
        ck2.close()
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_replica_restores_a_replaced_nodes_shard(tmp_path, _isolated_shm):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 4, port, str(tmp_path), _isolated_shm, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for f in glob.glob(f"/dev/shm/dwamd_{_isolated_shm}*"):
        os.remove(f)
    assert res == [(r, True) for r in range(4)], res


def _stress_worker(rank, world, port, root, prefix, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", LOCAL_WORLD_SIZE="1", NODE_RANK=str(rank),
                      DWAMD_SHM_PREFIX=f"{prefix}n{rank}")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.common.multi_process import SharedMemory
        from dlrover_wuqiong_amd.common.serialize import restricted_loads
        from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
        from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer
        from dlrover_wuqiong_amd.flash_checkpoint.layout import tensors_from_payload
        from dlrover_wuqiong_amd.flash_checkpoint.replica import _HDR

        import numpy as np

        ck = DdpCheckpointer(os.path.join(root, "ck"), replica_count=2)
        rm = ck.engine._replica_manager
        rm.chunk = 256 << 10  # many small chunks: transfers overlap the saves that follow
        base = torch.arange(2_000_000, dtype=torch.float32) + 1000 * rank
        last = 16
        saved = 0
        for step in range(1, last + 1):  # back-to-back saves while earlier ones replicate
            # a save finding both slots busy (one pinned by an outgoing
            # replica, the other still flushing) is skipped, on every rank
            if ck.save_checkpoint(step, {"w": base + step, "step": step}, storage_type=StorageType.MEMORY):
                saved = step
        last = saved
        ck.wait_latest_checkpoint()
        rm.wait()
        dist.barrier()
        peer = rm.backup_ranks[1 - rm.backup_ranks.index(rank)]
        seg = SharedMemory(f"replica_{peer}")
        hdr = np.frombuffer(seg.buf, dtype=np.int64, count=3)
        s_step, n, m = int(hdr[0]), int(hdr[1]), int(hdr[2])
        del hdr
        meta = restricted_loads(bytes(seg.buf[_HDR + n: _HDR + n + m]))
        w = tensors_from_payload(meta["tree"], seg.buf, _HDR)["model_states"]["w"].clone()
        ok = last > 0 and s_step == last and torch.equal(w, torch.arange(2_000_000, dtype=torch.float32) + 1000 * peer + s_step)
        del w
        seg.close()
        q.put((rank, bool(ok), rm.coalesced))
        dist.barrier()
        ck.close()
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e), 0))
    finally:
        dist.destroy_process_group()


def test_replica_consistent_under_continuous_saves(tmp_path, _isolated_shm):
    """Saves keep alternating the 2 shm slots while backups stream: every
    replica must hold exactly the bytes of the step it claims (no torn copy),
    the newest step must arrive, and stale tickets are coalesced."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_stress_worker, args=(r, 4, port, str(tmp_path), _isolated_shm, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for f in glob.glob(f"/dev/shm/dwamd_{_isolated_shm}*"):
        os.remove(f)
    assert [(r, ok) for r, ok, _ in res] == [(r, True) for r in range(4)], res
