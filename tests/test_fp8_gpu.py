"""FP8 kernels and Fp8Linear on the GPU vs the fp32 / torch-float8 reference
of the same op (ops/fp8.py, csrc/kernels/fp8.hip)."""

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd._native import kernels
    from dlrover_wuqiong_amd.ops import fp8

    kernels(required=True)
    fp8._STATES.clear()
    fp8._DEFAULTS.clear()
    yield
    fp8._STATES.clear()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("fmt", ["e4m3", "e5m2"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n", [8 * 4099, 1000 + 5])
def test_cast_kernel_matches_torch(fmt, dtype, n):
    from dlrover_wuqiong_amd.ops import fp8

    torch.manual_seed(n)
    st = fp8.fp8_state("cuda")
    i = st.register(fmt)
    st.scale[i] = 37.5  # values beyond the format's range saturate
    x = (torch.randn(n, device="cuda") * 8).to(dtype)
    x8 = fp8.cast_to_fp8(x, st, i, fmt)
    lim = fp8.FP8_MAX[fmt]
    ref = (x.float() * 37.5).clamp(-lim, lim).to(x8.dtype)
    same = (x8.view(torch.uint8) == ref.view(torch.uint8)).float().mean().item()
    assert same > 0.999, same
    assert st.amax_bits[i].view(torch.float32).item() == x.float().abs().max().item()


@pytest.mark.parametrize("fmt", ["e4m3", "e5m2"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(8192, 1600), (96, 200), (48, 64)])
def test_cast_transpose_kernel_matches_torch(fmt, dtype, shape):
    """dw_fp8_cast_t: both layouts from one pass (partial edge tiles
    included) equal torch's scale -> clamp -> cast, and the amax matches."""
    from dlrover_wuqiong_amd.ops import fp8

    torch.manual_seed(shape[0])
    st = fp8.fp8_state("cuda")
    i = st.register(fmt)
    st.scale[i] = 3.0
    x = (torch.randn(*shape, device="cuda") * 40).to(dtype)
    x8, x8t = fp8.cast_to_fp8_t(x, st, i, fmt)
    lim = fp8.FP8_MAX[fmt]
    ref = (x.float() * 3.0).clamp(-lim, lim).to(x8.dtype)
    assert (x8.view(torch.uint8) == ref.view(torch.uint8)).float().mean().item() > 0.999
    assert x8t.shape == (shape[1], shape[0]) and x8t.is_contiguous()
    assert torch.equal(x8t.view(torch.uint8), x8.view(torch.uint8).t())
    assert st.amax_bits[i].view(torch.float32).item() == x.float().abs().max().item()
    _r, only_t = fp8.cast_to_fp8_t(x, st, i, fmt, row=False)
    assert _r is None and torch.equal(only_t.view(torch.uint8), x8t.view(torch.uint8))


def test_update_scales_kernel():
    from dlrover_wuqiong_amd.ops import fp8

    st = fp8.fp8_state("cuda", history_len=3)
    idx = [st.register("e4m3"), st.register("e5m2"), st.register("e4m3")]
    for amax in ([2.0, 100.0, 0.0], [8.0, 1.0, 0.0]):
        st.amax_bits[: 3] = torch.tensor(amax, device="cuda").view(torch.int32)
        st.update()
    torch.cuda.synchronize()
    assert st.scale[idx[0]].item() == pytest.approx(448.0 / 8.0)
    assert st.scale[idx[1]].item() == pytest.approx(57344.0 / 100.0)
    assert st.scale[idx[2]].item() == 1.0  # never seen a value: unchanged
    assert st.inv_scale[idx[0]].item() == pytest.approx(8.0 / 448.0)
    assert int(st.amax_bits[:3].abs().sum()) == 0


@pytest.mark.parametrize("fmt", ["HYBRID", "E4M3"])
def test_fp8_linear_vs_linear(fmt):
    from dlrover_wuqiong_amd.ops import fp8

    torch.manual_seed(0)
    ref = nn.Linear(256, 512, device="cuda", dtype=torch.bfloat16)
    lin = nn.Linear(256, 512, device="cuda", dtype=torch.bfloat16)
    lin.load_state_dict(ref.state_dict())
    f8 = fp8.Fp8Linear(lin, fmt)
    for step in range(3):
        x = torch.randn(8, 64, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        xr = x.detach().clone().requires_grad_()
        y, yr = f8(x), ref(xr)
        g = torch.randn_like(yr)
        y.backward(g)
        yr.backward(g)
        assert torch.isfinite(y.float()).all() and y.dtype == torch.bfloat16
        assert _rel(y, yr) < 0.08, (step, _rel(y, yr))
        assert _rel(x.grad, xr.grad) < 0.15, (step, _rel(x.grad, xr.grad))
        assert _rel(lin.weight.grad, ref.weight.grad) < 0.15, step
        lin.weight.grad = lin.bias.grad = ref.weight.grad = ref.bias.grad = None
        fp8.fp8_update()


def test_auto_accelerate_fp8_gpt2_trains():
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.ops import fp8

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    model = GPT2(cfg)
    ok, res, _ = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": 3e-3},
                                 load_strategy=[("amp_native", {"dtype": torch.bfloat16}), "fp8"])
    assert ok and sum(isinstance(m, fp8.Fp8Linear) for m in res.model.modules()) > 0
    data = torch.randint(0, cfg.vocab_size, (8, 65), device="cuda")
    losses = []
    for _ in range(20):
        loss = res.model(data[:, :-1], data[:, 1:])
        loss.backward()
        res.optim.step()
        res.optim.zero_grad()
        losses.append(float(loss))
    assert all(map(lambda v: v == v, losses)) and losses[-1] < losses[0] - 0.5, losses


@pytest.mark.parametrize("fmt", ["e4m3", "e5m2"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_cast_keeps_nan_and_records_inf_amax(fmt, dtype):
    """A NaN input stays NaN in both cast kernels (fmaxf / fminf would turn
    it into -fmax), +-inf saturates, and the recorded amax is +inf so the
    next delayed-scaling update backs off -- the same as the CPU path."""
    from dlrover_wuqiong_amd.ops import fp8

    st = fp8.fp8_state("cuda")
    i = st.register(fmt)
    x = torch.randn(256, 64, device="cuda").to(dtype)
    x[3, 5] = float("nan")
    x[7, 9] = float("inf")
    x[100, 63] = -float("inf")
    lim = fp8.FP8_MAX[fmt]
    for cast in ("flat", "t"):
        st.amax_bits.zero_()
        if cast == "flat":
            x8 = fp8.cast_to_fp8(x, st, i, fmt).float().view(256, 64)
            x8t = None
        else:
            x8, x8t = fp8.cast_to_fp8_t(x, st, i, fmt)
            x8, x8t = x8.float(), x8t.float()
        assert torch.isnan(x8[3, 5]) and x8[7, 9].item() == lim and x8[100, 63].item() == -lim
        assert torch.isnan(x8).sum().item() == 1
        if x8t is not None:
            assert torch.isnan(x8t[5, 3]) and torch.isnan(x8t).sum().item() == 1
        assert st.amax_bits[i].view(torch.float32).item() == float("inf")
    cpu_st = fp8.Fp8State(torch.device("cpu"))
    j = cpu_st.register(fmt)
    ref = fp8.cast_to_fp8(x.cpu(), cpu_st, j, fmt)
    assert torch.equal(torch.isnan(ref.float()), torch.isnan(x8.cpu()))
    assert cpu_st.amax_bits[j].view(torch.float32).item() == float("inf")


def test_fp8_linear_propagates_nan():
    from dlrover_wuqiong_amd.ops import fp8

    torch.manual_seed(0)
    lin = nn.Linear(256, 512, device="cuda", dtype=torch.bfloat16)
    f8 = fp8.Fp8Linear(lin, "HYBRID")
    x = torch.randn(4, 64, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    with torch.no_grad():
        x[0, 0, 0] = float("nan")
    y = f8(x)
    assert torch.isnan(y.float()).any()
    y.float().sum().backward()
    assert not torch.isfinite(lin.weight.grad.float()).all()
