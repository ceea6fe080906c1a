"""xpu_timer native HIP-event backend on the GPU: per-shape GEMM timing and
device-hang detection (a calibrated ~2 s spin kernel vs a 0.5 s timeout)."""

import time

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_gemm_timing_and_hang_detection():
    from dlrover_wuqiong_amd.utils.xpu_timer import XpuTimer, _HipBackend

    hangs = []
    t = XpuTimer(hang_timeout=0.5, poll_ms=10, on_hang=[lambda d, s: hangs.append(d)]).install(collectives=False)
    try:
        assert isinstance(t.backend, _HipBackend)
        a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
        for _ in range(20):
            torch.mm(a, b)
        torch.cuda.synchronize()
        assert t.flush(10)
        st = {s.key: s for s in t.stats()}["mm|4096_4096_4096"]
        assert st.count == 20 and st.avg_us > 0
        assert 50 < st.rate()["tflops"] < 2600, st  # plausible for MI355X bf16
        # calibrate torch.cuda._sleep, then spin ~2 s inside a timed region
        s0 = time.time()
        torch.cuda._sleep(10_000_000)
        torch.cuda.synchronize()
        per_cycle = max(time.time() - s0, 1e-4) / 10_000_000
        cycles = int(min(2.0 / per_cycle, 2e10))
        with t.timed("spin|x", 0.0, a):
            torch.cuda._sleep(cycles)
        deadline = time.time() + 5
        while not hangs and time.time() < deadline:
            time.sleep(0.05)
        torch.cuda.synchronize()
        assert hangs and "spin|x" in hangs[0]
        time.sleep(0.2)
        assert t.hang_status()[0] == 0  # cleared once the op finished
    finally:
        t.uninstall()


def test_framework_kernels_are_timed():
    """The framework's own HIP launches (attention, norms, fused Adam, ...)
    appear as ``kernel|dw_*`` records next to the torch GEMMs."""
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams
    from dlrover_wuqiong_amd.utils.xpu_timer import XpuTimer

    t = XpuTimer(hang_timeout=60, poll_ms=10).install(collectives=False)
    try:
        torch.manual_seed(0)
        with torch.device("cuda"):
            model = GPT2(GPT2Config.named("gpt2-tiny"))
        model.to(torch.bfloat16)
        flat = FlatParams(model)
        opt = FusedAdamW(flat, lr=1e-3)
        x = torch.randint(0, 1024, (2, 129), device="cuda")
        for _ in range(3):
            model(x[:, :-1], x[:, 1:]).backward()
            opt.step()
            flat.zero_grad()
        torch.cuda.synchronize()
        assert t.flush(10)
        st = {s.key: s for s in t.stats()}
        kern = {k: s for k, s in st.items() if k.startswith("kernel|")}
        assert any("attn_fwd" in k for k in kern) and any("attn_bwd" in k for k in kern), sorted(st)
        assert any("adam" in k.lower() for k in kern), sorted(kern)
        assert all(s.count > 0 and s.avg_us > 0 for s in kern.values())
        assert "kind=\"kernel\"" in t.prometheus_text()
    finally:
        t.uninstall()
