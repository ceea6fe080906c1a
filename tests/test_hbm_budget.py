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
