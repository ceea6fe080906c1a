"""ATorch data utilities: shared-memory batch ring (broadcast to a model-
parallel group, coworker work queue), GPU preloader, unordered loader,
master-sharded elastic dataset (parity: ATorch tests/data)."""

import os

import pytest
import torch
import torch.multiprocessing as mp
from torch.utils.data import DataLoader, Dataset


class _Seq(Dataset):
    def __init__(self, n=37):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return {"ids": torch.full((4,), i, dtype=torch.int64), "x": torch.randn(3) * 0 + i, "tag": "s"}


def _mp_rank(rank, group, prefix, q):
    try:
        from dlrover_wuqiong_amd.atorch.data import ShmDataLoader

        dl = ShmDataLoader(_Seq(), {"batch_size": 5, "num_workers": 1 if rank == 0 else 0}, rank=rank,
                           group_size=group, shm_name_prefix=prefix, shm_data_size=3)
        seen = []
        for _epoch in range(2):
            ep = []
            for b in dl:
                assert b["tag"] == ["s"] * len(b["ids"])
                ep.append(b["ids"][:, 0].tolist())
            seen.append(ep)
        q.put((rank, len(dl), seen))
        dl.close()
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, -1, traceback.format_exc() + repr(e)))


def test_shm_dataloader_broadcasts_same_batches():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    prefix = f"t{os.getpid()}"
    ps = [ctx.Process(target=_mp_rank, args=(r, 3, prefix, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = {r: (n, s) for r, n, s in (q.get(timeout=120) for _ in ps)}
    for p in ps:
        p.join(30)
    expect = [list(range(i, min(i + 5, 37))) for i in range(0, 37, 5)]
    for r in range(3):
        assert res[r][0] == 8, res[r]
        assert res[r][1] == [expect, expect], (r, res[r][1])


def _coworker(cw, prefix, q):
    from dlrover_wuqiong_amd.atorch.data import coworker_produce

    q.put(("cw", cw, coworker_produce(_Seq(40), {"batch_size": 4}, cw, 2, shm_name_prefix=prefix,
                                      shm_data_size=4, process_fn=lambda b: {"ids": b["ids"] * 10})))


def _worker(w, prefix, q):
    from dlrover_wuqiong_amd.atorch.data import ShmDataLoader

    dl = ShmDataLoader(None, {}, coworker=True, shm_name_prefix=prefix)
    got = [b["ids"][:, 0].tolist() for b in dl]
    q.put(("w", w, got))
    dl.close()


def test_coworker_shared_ring_distributes_batches():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    prefix = f"cw{os.getpid()}"
    ps = [ctx.Process(target=_coworker, args=(c, prefix, q)) for c in range(2)]
    ps += [ctx.Process(target=_worker, args=(w, prefix, q)) for w in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(30)
    produced = sum(n for k, _, n in res if k == "cw")
    batches = [b for k, _, got in res if k == "w" for b in got]
    assert produced == 10 and len(batches) == 10
    assert sorted(v for b in batches for v in b) == [10 * i for i in range(40)]


def test_gpu_preloader_and_unordered_cpu():
    from dlrover_wuqiong_amd.atorch.data import GpuPreLoader, UnorderedDataLoader

    pre = GpuPreLoader(DataLoader(_Seq(10), batch_size=4), device="cpu",
                       post_processing=lambda b: {**b, "ids": b["ids"] + 1})
    got = [b["ids"][:, 0].tolist() for b in pre]
    assert got == [[1, 2, 3, 4], [5, 6, 7, 8], [9, 10]] and len(pre) == 3 and pre.batch_size == 4
    ul = UnorderedDataLoader(_Seq(20), batch_size=5, num_workers=2)
    vals = sorted(v for b in ul for v in b["ids"][:, 0].tolist())
    assert vals == list(range(20))


class _SlowFirst(torch.utils.data.Dataset):
    def __len__(self):
        return 24

    def __getitem__(self, i):
        if i == 0:
            import time

            time.sleep(1.5)
        if i == 13 and getattr(self, "fail", False):
            raise ValueError("bad sample 13")
        return torch.tensor([i])


def test_unordered_loader_completion_order_and_errors():
    """A slow sample delays only its own batch; every batch arrives exactly
    once; the other workers keep draining the shared queue; a worker
    exception re-raises in the main process."""
    from dlrover_wuqiong_amd.atorch.data import UnorderedDataLoader

    ul = UnorderedDataLoader(_SlowFirst(), batch_size=2, num_workers=3)
    order = [b[:, 0].tolist() for b in ul]
    assert sorted(v for b in order for v in b) == list(range(24))
    assert order[0] != [0, 1] and order.index([0, 1]) >= 6  # not head-of-line blocked
    per = ul.stats()
    assert sum(per) == 12 and max(per) >= 5  # the slow worker produced 1; the others took the rest
    # in-order torch DataLoader for contrast: batch 0 comes first, after the sleep
    ref = [b[:, 0].tolist() for b in DataLoader(_SlowFirst(), batch_size=2, num_workers=3)]
    assert ref[0] == [0, 1]
    bad = _SlowFirst()
    bad.fail = True
    with pytest.raises(RuntimeError, match="bad sample 13"):
        for _ in UnorderedDataLoader(bad, batch_size=2, num_workers=2):
            pass


def test_elastic_dataset_from_master():
    from dlrover_wuqiong_amd.atorch.data import SimpleElasticDataset
    from dlrover_wuqiong_amd.elastic_agent.master_client import MasterClient
    from dlrover_wuqiong_amd.master.master import JobMaster

    m = JobMaster(port=0, node_num=1, loop_interval=0.2)
    m.start_background()
    try:
        c = MasterClient(m.addr, node_id=0, retries=2, retry_interval=0.1)
        ds = SimpleElasticDataset("eds", lambda i: i * 2, dataset_size=24, batch_size=4, epochs=1,
                                  master_client=c)
        assert len(ds) == 24
        vals = []
        for _ in range(24):
            vals.append(ds[0])
            if len(vals) % 4 == 0:
                ds.report_batch_done(4)
        assert sorted(vals) == [2 * i for i in range(24)]
        with pytest.raises(IndexError):
            ds[0]
    finally:
        m.stop()


@pytest.mark.gpu
def test_shm_ring_direct_dma_to_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd.atorch.data.shm_ring import BROADCAST, ShmBatchRing

    name = f"dwgpu_ring_{os.getpid()}"
    w = ShmBatchRing(name, True, nslots=2, slot_bytes=1 << 22, nreaders=1, mode=BROADCAST)
    r = ShmBatchRing(name, False)
    try:
        for i in range(5):
            w.put({"a": torch.arange(100000) + i, "b": torch.full((7, 9), float(i), dtype=torch.bfloat16)})
            b = r.get(0, device="cuda")
            assert b["a"].is_cuda and torch.equal(b["a"].cpu(), torch.arange(100000) + i)
            assert torch.equal(b["b"].cpu(), torch.full((7, 9), float(i), dtype=torch.bfloat16))
        w.stop()
        assert r.get(0, device="cuda") is None
    finally:
        r.close()
        w.close()
