"""BF16 grad scalers, sparse all-reduce (2-rank gloo), network counter
monitor (fake sysfs), trace analysis (compute/communication overlap) and
the FLOPs profiler.  Parity: reference atorch/utils/{grad_scaler,sparse,
ib_monitor,parse_trace_json,prof}.py and their tests."""

import json
import os

import torch

from dlrover_wuqiong_amd.common.rpc import find_free_port


def test_bf16_grad_scaler_skips_overflow():
    from dlrover_wuqiong_amd.atorch.utils.grad_scaler import BF16GradScaler

    p = torch.nn.Parameter(torch.ones(4))
    opt = torch.optim.SGD([p], lr=0.1)
    s = BF16GradScaler()
    loss = (p * 2).sum()
    s.scale(loss).backward()
    s.step(opt)
    s.update()
    assert not s.has_overflow() and torch.allclose(p.detach(), torch.full((4,), 0.8))
    assert s.get_scale() == 1.0
    opt.zero_grad()
    (p * float("inf")).sum().backward()
    s.step(opt)
    s.update()
    assert s.has_overflow() and torch.allclose(p.detach(), torch.full((4,), 0.8))
    assert s.get_scale() == 1.0


def _sparse_worker(rank, world, port, q):
    import torch.distributed as dist

    from dlrover_wuqiong_amd.atorch.utils.sparse import all_reduce_sparse

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dense = torch.zeros(6, 3)
        dense[rank] = rank + 1.0
        dense[5] = 1.0
        if rank == 1:
            dense[3] = 2.0
        out = all_reduce_sparse(dense.to_sparse())
        q.put((rank, out.to_dense().tolist()))
    finally:
        dist.destroy_process_group()


def test_all_reduce_sparse_two_ranks():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    ps = [ctx.Process(target=_sparse_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
    exp = torch.zeros(6, 3)
    exp[0], exp[1], exp[3], exp[5] = 1.0, 2.0, 2.0, 2.0
    for _, d in res:
        assert torch.equal(torch.tensor(d), exp)


def test_net_monitor_fake_sysfs(tmp_path):
    from dlrover_wuqiong_amd.utils.net_monitor import NetStat

    c = tmp_path / "infiniband" / "mlx5_0" / "ports" / "1" / "counters"
    c.mkdir(parents=True)
    e = tmp_path / "net" / "eth0" / "statistics"
    e.mkdir(parents=True)

    def write(tx, rx, etx, erx):
        (c / "port_xmit_data").write_text(str(tx))
        (c / "port_rcv_data").write_text(str(rx))
        (e / "tx_bytes").write_text(str(etx))
        (e / "rx_bytes").write_text(str(erx))

    ns = NetStat(sysfs_root=str(tmp_path))
    write(0, 0, 0, 0)
    ns.sample(now=10.0)
    write(250_000_000, 500_000_000, 1_000_000_000, 0)
    r = ns.sample(now=12.0)
    assert abs(r["mlx5_0:1"]["tx_gbps"] - 0.5) < 1e-9 and abs(r["mlx5_0:1"]["rx_gbps"] - 1.0) < 1e-9
    assert abs(r["eth0"]["tx_gbps"] - 0.5) < 1e-9
    assert ns.snapshot()["eth0"]["rx_gbps"] == 0.0


def test_trace_analysis_overlap(tmp_path):
    from dlrover_wuqiong_amd.utils import trace_analysis as ta

    ev = [
        {"ph": "X", "cat": "kernel", "name": "Cijk_Ailk_Bljk_BBS", "ts": 0, "dur": 100},
        {"ph": "X", "cat": "kernel", "name": "ncclDevKernel_AllReduce_Sum_bf16_RING_LL", "ts": 50, "dur": 100},
        {"ph": "X", "cat": "kernel", "name": "attn_fwd_kernel<64>", "ts": 160, "dur": 40},
        {"ph": "X", "cat": "cpu_op", "name": "aten::mm", "ts": 0, "dur": 500},
    ]
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"traceEvents": ev}))
    r = ta.analyze(ta.load(str(p)))
    assert r["kernels"] == 3
    assert abs(r["comm_s"] - 100e-6) < 1e-12 and abs(r["exposed_comm_s"] - 50e-6) < 1e-12
    assert abs(r["overlap_pct"] - 50.0) < 1e-6
    assert abs(r["idle_s"] - 10e-6) < 1e-12
    assert set(r["by_category_s"]) == {"gemm", "communication", "attention"}
    csvp = tmp_path / "k.csv"
    csvp.write_text("Kernel_Name,Start_Timestamp,End_Timestamp\nrcclAllGather,0,1000\nCijk_x,500,2000\n")
    r2 = ta.analyze(ta.load(str(csvp)))
    assert abs(r2["overlap_pct"] - 50.0) < 1e-6


def test_aprofiler_flops():
    from dlrover_wuqiong_amd.atorch.utils.prof import AProfiler, flash_attn_flops

    m = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 32))
    x = torch.randn(16, 64)
    prof = AProfiler(m)
    prof.start_profile()
    m(x).sum().backward()
    prof.stop_profile()
    fwd = 2 * 16 * 64 * 128 + 2 * 16 * 128 * 32
    # forward + backward (dgrad of the second linear, wgrads of both; the
    # first layer's input needs no gradient)
    assert prof.get_total_flops() == fwd + 2 * 16 * 64 * 128 + 2 * 2 * 16 * 128 * 32
    assert prof.get_total_params() == 64 * 128 + 128 + 128 * 32 + 32
    assert prof.get_total_duration() > 0 and prof.mfu() is not None
    lines = prof.print_model_profile()
    assert "total:" in lines[-1]
    assert flash_attn_flops((1, 1024, 8, 64), causal=True) == 4 * 8 * 1024 * 1024 * 64 // 2
