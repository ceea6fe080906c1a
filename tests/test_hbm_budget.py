"""HBM-budget preflight of the flash-checkpoint data path (hbm_budget.py) for
the N=8 configurations the driver runs on a whole MI355X node, with mocked
``mem_get_info``: staging (double / single / ring), deep vs import standby,
and the bounded restore all-gather temporary -- and the copier's own
decisions follow the same rules."""

import pytest
import torch

from dlrover_wuqiong_amd.flash_checkpoint import hbm_budget as hb

GiB = 1 << 30
HBM = 288 * GiB  # MI355X


def test_gpt2_1p5b_ddp_n8():
    # per GPU: bf16 params + grads, fp32 master + Adam (24.9 GB state),
    # activations of B=8 x S=1024 on top; 21.8 GB replicated payload split 8 ways
    p = hb.plan(HBM, worker_state=int(24.9 * GiB), worker_peak=80 * GiB, payload=int(21.8 * GiB),
                world_local=8, replicated=True, standby="deep")
    assert p.fits and p.standby == "deep" and p.staging == "double"
    assert p.slice_bytes == -(-int(21.8 * GiB) // 8)
    assert p.staging_bytes == 2 * p.slice_bytes
    # the whole-payload temporary (21.8 GB) would exceed the 16 GiB gather
    # cap: the restore gathers in rounds of 8 x chunk
    assert p.gather_temp_bytes <= 16 * GiB and p.gather_chunk < p.slice_bytes
    assert "gather" in p.notes
    d = p.as_dict()
    assert d["staging"] == "double" and d["restore_peak_gib"] < 288


def test_gpt2_1p5b_ddp_n1_one_round():
    p = hb.plan(HBM, worker_state=int(24.9 * GiB), worker_peak=80 * GiB, payload=int(21.8 * GiB),
                world_local=1, replicated=True, standby="import")
    assert p.fits and p.gather_temp_bytes == 0 and p.staging == "double"
    # the import standby caches about the worker's peak next to it
    assert 0 < p.standby_bytes <= 80 * GiB


def test_llama3_8b_fsdp_n8():
    # FSDP: every rank owns a shard (no gather); 8B params -> ~16 GB state
    # per rank, ~14 GB checkpoint shard, activations at seq 4096
    p = hb.plan(HBM, worker_state=16 * GiB, worker_peak=70 * GiB, payload=14 * GiB, world_local=8,
                replicated=False, standby="deep")
    assert p.fits and p.staging == "double" and p.standby == "deep"
    assert p.slice_bytes == 14 * GiB and p.gather_temp_bytes == 0


def test_llama3_70b_tp8_shard_falls_back():
    # Megatron TP=8 rank shard of 70B: 123.5 GB checkpoint, 132 GB peak;
    # a deep standby (another ~124 GB) cannot fit next to it + one slice
    p = hb.plan(HBM, worker_state=124 * GiB, worker_peak=132 * GiB, payload=int(123.5 * GiB), world_local=8,
                replicated=False, standby="deep")
    assert p.standby == "import" and "standby" in p.notes
    assert p.staging == "single" and p.fits
    # a larger activation peak leaves no room for even one slice: ring
    q = hb.plan(HBM, worker_state=124 * GiB, worker_peak=160 * GiB, payload=int(123.5 * GiB), world_local=8,
                replicated=False, standby="import")
    assert q.staging == "ring" and q.staging_bytes <= 4 * GiB


def test_gather_chunk_rules():
    assert hb.gather_chunk(2 * GiB, 8, free=200 * GiB) == 2 * GiB  # 16 GiB total: one round
    c = hb.gather_chunk(int(2.7 * GiB), 8, free=200 * GiB)
    assert c * 8 <= 16 * GiB and c % (2 << 20) == 0
    assert hb.gather_chunk(int(2.7 * GiB), 8, free=10 * GiB) * 8 <= 6 * GiB + 8 * (64 << 20)
    assert hb.gather_chunk(GiB, 1, free=0) == GiB  # no gather


def test_copier_decisions_follow_the_budget(monkeypatch):
    from dlrover_wuqiong_amd.flash_checkpoint.copier import GpuCopier

    free = {"v": 100 * GiB}
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a: (free["v"], HBM))
    c = GpuCopier.__new__(GpuCopier)  # sizing logic only: no device needed
    c.device, c._stagings, c._nbuf, c.staging_reserve = "cuda", [None, None], 0, 24 * GiB
    c._decide_buffers(30 * GiB)
    assert c._nbuf == hb.staging_buffers(100 * GiB, 0, 30 * GiB, 24 * GiB) == 2
    c._nbuf = 0
    free["v"] = 70 * GiB
    c._decide_buffers(30 * GiB)
    assert c._nbuf == 1
    c.staging_mode, c._ring_decision, c._ext = "auto", None, None
    c.ring_slots, c.ring_chunk, c.ring_hbm, c._ring_auto = 4, GiB, 0, 0
    free["v"] = 40 * GiB
    c._stagings = [None, None]
    c.wait = lambda: None
    assert c._use_ring(30 * GiB) is hb.use_ring(40 * GiB, 0, 30 * GiB, 24 * GiB) is True


def test_copier_counts_the_allocator_cache_as_free(monkeypatch):
    """A recovered import worker holds its standby's reservation in the
    caching allocator: the driver reports little free HBM, but the staging
    decision must count the cached blocks (else it picks one buffer or the
    ring and every later save waits on the flush)."""
    from dlrover_wuqiong_amd.flash_checkpoint.copier import GpuCopier, device_free_bytes

    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a: (10 * GiB, HBM))
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda *a: 130 * GiB)
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda *a: 40 * GiB)
    assert device_free_bytes("cuda") == 100 * GiB
    c = GpuCopier.__new__(GpuCopier)
    c.device, c._stagings, c._nbuf, c.staging_reserve = "cuda", [None, None], 0, 24 * GiB
    c._decide_buffers(30 * GiB)
    assert c._nbuf == 2
    c.staging_mode, c._ring_decision, c._ext = "auto", None, None
    c.ring_slots, c.ring_chunk, c.ring_hbm, c._ring_auto = 4, GiB, 0, 0
    c.wait = lambda: None
    c._refresh_external = lambda n: None
    assert c._use_ring(30 * GiB) is False


def test_n8_restart_allocation_plan():
    """GPT2-1.5B DDP on 8 GPUs (replicated 21.8 GB state, 1/8 slices): every
    byte the restart path needs is held by the standby -- the gather
    temporary it reserves equals what copier.restore would allocate, and the
    plan fits next to the live worker on a 288 GB card, tier on and off."""
    from dlrover_wuqiong_amd.flash_checkpoint import prewarm

    payload = int(21.8 * GiB)
    state, peak = int(24.9 * GiB), int(45.5 * GiB)
    per = -(-payload // 8)
    for standby in ("deep", "import"):
        for tier in (True, False):
            p = hb.plan(HBM, worker_state=state, worker_peak=peak, payload=payload, world_local=8, replicated=True,
                        standby=standby, hbm_tier=tier)
            assert p.fits and p.staging == "double", (standby, tier, p)
            assert p.gather_temp_bytes == hb.gather_chunk(per, 8, 1 << 62) * 8 <= 16 * GiB + 8 * (2 << 20)
            assert p.standby_bytes >= p.gather_temp_bytes
            if standby == "import" and not tier:
                assert p.standby_bytes >= 2 * per  # its own staging buffers
    # what the parked standby reserves (prewarm.restore_temp_bytes) is that temporary
    prewarm._STATE_BYTES["seg"], prewarm._NSLICES["seg"] = payload, 8
    try:
        assert prewarm.restore_temp_bytes() == p.gather_temp_bytes
    finally:
        prewarm._STATE_BYTES.pop("seg"), prewarm._NSLICES.pop("seg")


@pytest.mark.parametrize("per,world,chunk", [(1000, 4, 1000), (1000, 4, 256), (999, 3, 100)])
def test_chunked_gather_scatter_plan_covers_payload(per, world, chunk):
    """The restore's per-round scatter descriptors (copier.restore) place
    every payload byte exactly once (pure-index model of the loop)."""
    payload = per * world - 7
    pieces = [(0, 10_000, 300), (300, 20_000, per * world - 300 - 7)]  # (payload_off, dst, n)
    dst_of = {}
    for o in range(0, per, chunk):
        n = min(chunk, per - o)
        for r in range(world):
            a, b = r * per + o, r * per + o + n
            for off, dst, m in pieces:
                x0, x1 = max(a, off), min(b, off + m)
                for x in range(x0, x1):
                    assert x not in dst_of
                    dst_of[x] = dst + (x - off)
    assert sorted(dst_of) == list(range(payload))


# ----------------------------------------------------- node host-memory plan
def _mi(total_gib, avail_gib):
    return {"MemTotal": int(total_gib * GiB), "MemAvailable": int(avail_gib * GiB)}


def test_host_plan_gpt2_1p5b_ddp_n8_two_slots():
    # replicated: ONE node segment (the 8 ranks write 1/8 slices of it)
    p = hb.host_plan(int(21.8 * GiB), segments=1, shm_free=1000 * GiB, meminfo=_mi(2048, 1900), reserve=64 * GiB)
    assert p.fits and p.slots == 2 and not p.notes
    assert p.need_bytes >= 2 * int(21.8 * GiB)
    d = p.as_dict()
    assert d["slots"] == 2 and d["need_bytes_gib"] >= 43.6


def test_host_plan_llama3_8b_fsdp_n8():
    # FSDP: one segment per rank, 1/8 of bf16 params + fp32 master + Adam (16 B/param)
    shard = int(8.03e9 * 16 / 8)
    p = hb.host_plan(shard, segments=8, shm_free=1000 * GiB, meminfo=_mi(2048, 1900), reserve=64 * GiB)
    assert p.fits and p.slots == 2
    # a node with 200 GiB of shm: one slot only
    p = hb.host_plan(shard, segments=8, shm_free=200 * GiB, meminfo=_mi(2048, 1900), reserve=64 * GiB)
    assert p.slots == 1 and "1 slot" in p.notes["slots"]


def test_host_plan_llama3_70b_tp8():
    shard = int(123.5 * GiB)  # per-rank TP=8 shard payload (profiles/megatron_llama3_70b_tp8_shard.log)
    # 8 x 2 x 123.5 GiB = 1976 GiB does not fit 1.5 TiB of shm, one slot does
    p = hb.host_plan(shard, segments=8, shm_free=1536 * GiB, meminfo=_mi(2048, 1900), reserve=64 * GiB)
    assert p.fits and p.slots == 1
    assert p.pin_sec_est > 40  # ~46 s measured for one 123.5 GB shard's first pinning
    # a node whose MemAvailable (not tmpfs size) is the limit
    p = hb.host_plan(shard, segments=8, shm_free=4096 * GiB, meminfo=_mi(1024, 900), reserve=64 * GiB)
    assert not p.fits and p.slots == 0 and "only" in p.notes["slots"]
    # this job's old segments are replaced, so their pages count as room
    p = hb.host_plan(shard, segments=8, shm_free=4096 * GiB, meminfo=_mi(1024, 900), reserve=64 * GiB,
                     reclaimable=8 * shard)
    assert p.fits and p.slots == 1


def test_host_plan_reads_statvfs_and_meminfo(monkeypatch, tmp_path):
    import collections

    mi = tmp_path / "meminfo"
    mi.write_text("MemTotal:       65536000 kB\nMemAvailable:   32768000 kB\nShmem: 10 kB\n")
    vfs = collections.namedtuple("vfs", "f_bavail f_frsize")
    monkeypatch.setattr(hb.os, "statvfs", lambda p: vfs(10 * (GiB // 4096), 4096))
    got = hb.read_meminfo(str(mi))
    assert got["MemAvailable"] == 32768000 * 1024 and got["MemTotal"] == 65536000 * 1024
    assert hb.shm_free_bytes() == 10 * GiB
    monkeypatch.setattr(hb, "read_meminfo", lambda path="/proc/meminfo": got)
    p = hb.host_plan(3 * GiB, segments=1)  # 2 x 3 GiB fits the 10 GiB tmpfs
    assert p.slots == 2 and p.shm_free == 10 * GiB
    p = hb.host_plan(7 * GiB, segments=1)
    assert p.slots == 1


def test_engine_creates_one_slot_segment_when_two_do_not_fit(tmp_path, monkeypatch):
    """End to end on CPU: the engine asks the plan before creating the
    segment; with room for one slot it creates a 1-slot segment, saves and
    restores through it (readers adopt the slot count from the header); with
    room for none it raises HostMemoryError instead of risking SIGBUS."""
    from dlrover_wuqiong_amd.flash_checkpoint import engine as eng_mod
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer

    real = hb.host_plan
    monkeypatch.setattr(hb, "host_plan", lambda payload, segments, want_slots=2, reclaimable=0, **kw: real(
        payload, segments, want_slots, shm_free=int(1.5 * payload) + (1 << 20), meminfo=_mi(1024, 1000),
        reserve=0, reclaimable=0))
    w = torch.nn.Linear(512, 512)
    ck = DdpCheckpointer(str(tmp_path / "ck"))
    assert ck.save_checkpoint(3, {"model": w.state_dict(), "step": 3}, storage_type=StorageType.MEMORY)
    ck.wait_latest_checkpoint()
    h = ck.engine._shm_handler
    assert h.num_slots == 1 and ck.engine.host_plan["slots"] == 1
    assert ck.save_checkpoint(4, {"model": w.state_dict(), "step": 4}, storage_type=StorageType.MEMORY)
    ck.wait_latest_checkpoint()
    sd = ck.load_checkpoint()
    assert sd["step"] == 4 and torch.equal(sd["model"]["weight"], w.weight)
    ck.close()
    monkeypatch.setattr(hb, "host_plan", lambda payload, segments, want_slots=2, reclaimable=0, **kw: real(
        payload, segments, want_slots, shm_free=1 << 20, meminfo=_mi(1024, 1000), reserve=0))
    ck2 = DdpCheckpointer(str(tmp_path / "ck2"))
    big = torch.nn.Linear(1024, 1024)  # a new size: the segment is re-created
    with pytest.raises(hb.HostMemoryError):
        ck2.save_checkpoint(5, {"model": big.state_dict(), "step": 5}, storage_type=StorageType.MEMORY)
    ck2.close()
    del eng_mod


def test_deferred_write_back_budget_70b_tp8(monkeypatch):
    """Llama-3-70B TP=8 shard (8.8e9 elements: bf16 params + fp32 master +
    Adam = 123.5 GB, bf16 gradient 17.6 GB) on a ring: the plan counts the
    kept gradients of the deferred steps, and the optimizer picks K from the
    free HBM at ring time -- the full 4 with room, fewer when tight, 0
    (wait for the ring) when not even one kept gradient fits."""
    import torch.nn as nn

    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    elems = int(8.8e9)
    grad = 2 * elems
    state = elems * (2 + 4 + 4 + 4) + grad
    p = hb.plan(HBM, worker_state=state, worker_peak=state + 30 * GiB, payload=elems * 14, world_local=8,
                replicated=False, standby="import", grad_bytes=grad, ring_chunk=GiB, ring_slots=64)
    assert p.staging == "ring" and p.defer_steps >= 1 and p.defer_bytes == p.defer_steps * grad
    assert "defer" in p.notes
    tight = hb.plan(HBM, worker_state=state, worker_peak=HBM - 65 * GiB, payload=elems * 14, world_local=8,
                    replicated=False, standby="import", grad_bytes=grad, ring_chunk=GiB, ring_slots=64)
    assert tight.staging == "ring" and tight.defer_steps == 0 and "wait" in tight.notes["defer"]

    opt = FusedAdamW(FlatParams(nn.Linear(8, 8)), lr=1e-3)
    per_step = grad  # the whole shard's gradient still unstaged (worst case)
    # the allocator's cache (the next forward's activations) is never counted
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda *a: 200 * GiB)
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda *a: 150 * GiB)
    for free, want in ((100 * GiB, 4), (40 * GiB, 2), (15 * GiB, 0)):
        monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a, f=free: (f, HBM))
        k = opt._defer_budget(per_step)
        assert k == want == opt.last_defer_plan["steps"], (free, k, opt.last_defer_plan)
        assert opt.last_defer_plan["decision"] == ("defer" if want else "wait")
