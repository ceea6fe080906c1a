"""Hang detection -> agent relaunch (worker heartbeat / relaunch request via the
agent control dir) and the xpu_timer CPU backend + Prometheus exporter
(parity: ATorch fault_tolerance/hanging_detector.py, dev/xpu_timer)."""

import os
import subprocess
import sys
import urllib.request

import torch

from conftest import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HANG_SCRIPT = r'''
import os, sys, time
from dlrover_wuqiong_amd.atorch.fault_tolerance import HangingDetector, heartbeat
restart = int(os.environ["TORCHELASTIC_RESTART_COUNT"])
mode = sys.argv[1]
det = HangingDetector(timeout=1.0, monitor_interval=0.1)
det.start()
for step in range(6):
    det.report_normal()
    time.sleep(0.05)
if restart == 0:
    if mode == "detector":
        time.sleep(600)          # hang: the in-process detector requests a relaunch
    else:
        det.stop(finalize=True)  # hang with the detector off: the agent's heartbeat timeout fires
        time.sleep(600)
with open(sys.argv[2], "a") as f:
    f.write(f"done restart={restart}\n")
'''


def _launch(tmp_path, mode, extra):
    script = tmp_path / "hang.py"
    script.write_text(HANG_SCRIPT)
    out = tmp_path / "out.txt"
    env = dict(os.environ, PYTHONPATH=REPO, DWAMD_WARM_STANDBY="0")
    p = subprocess.run([sys.executable, "-m", "dlrover_wuqiong_amd.trainer.run", "--nnodes", "1",
                        "--nproc-per-node", "1", "--max-restarts", "1"] + extra + [str(script), mode, str(out)],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=180)
    return p, out


def test_hanging_detector_requests_relaunch(tmp_path):
    p, out = _launch(tmp_path, "detector", [])
    assert p.returncode == 0, p.stdout[-3000:]
    assert "relaunch requested" in p.stdout
    assert out.read_text().strip() == "done restart=1"


def test_agent_heartbeat_timeout_relaunch(tmp_path):
    p, out = _launch(tmp_path, "agent", ["--relaunch-on-hang", "2"])
    assert p.returncode == 0, p.stdout[-3000:]
    assert "no heartbeat" in p.stdout
    assert out.read_text().strip() == "done restart=1"


def test_xpu_timer_cpu_backend_and_exporter():
    from dlrover_wuqiong_amd.utils.xpu_timer import XpuTimer

    t = XpuTimer(device="cpu").install(collectives=False)
    try:
        a, b = torch.randn(64, 32), torch.randn(32, 16)
        for _ in range(5):
            torch.mm(a, b)
        torch.nn.functional.linear(torch.randn(4, 8, 32), torch.randn(16, 32))
        with t.timed("all_reduce|float32|4096|ws2", 4096.0):
            pass
        stats = {s.key: s for s in t.stats()}
        assert stats["mm|64_16_32"].count == 5
        assert stats["linear|32_16_32"].count == 1
        assert stats["mm|64_16_32"].rate()["tflops"] > 0
        port = t.start_exporter(0)
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=10).read().decode()
        assert 'dwamd_xpu_timer_avg_latency_us{' in body and 'kind="mm",shape="64_16_32"' in body
        assert "dwamd_xpu_timer_busbw_gbps" in body and "dwamd_xpu_timer_hang" in body
        assert "mm|64_16_32" in t.report()
    finally:
        t.uninstall()
    # mode removed: no more records
    n = {s.key: s.count for s in t.stats()}["mm|64_16_32"]
    torch.mm(torch.randn(64, 32), torch.randn(32, 16))
    assert {s.key: s.count for s in t.stats()}["mm|64_16_32"] == n


def _coll_worker(rank, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from dlrover_wuqiong_amd.utils.xpu_timer import XpuTimer

    t = XpuTimer(device="cpu").install(gemm=False)
    x = torch.ones(1024)
    for _ in range(3):
        dist.all_reduce(x)
    keys = {s.key: s.count for s in t.stats()}
    t.uninstall()
    q.put((rank, keys.get("all_reduce|float32|4096|ws2", 0), float(x[0])))
    dist.destroy_process_group()


def test_xpu_timer_wraps_collectives():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_coll_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    assert res == [(0, 3, 8.0), (1, 3, 8.0)]
