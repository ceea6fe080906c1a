"""FP8 linear layers (ops/fp8.py) on the CPU execution path: delayed-scaling
bookkeeping, numerics vs nn.Linear, and the auto_accelerate ``fp8`` strategy
(parity: ATorch amp_optimization.py Fp8Optimization, Transformer Engine
te.Linear + DelayedScaling)."""

import pytest
import torch
import torch.nn as nn


@pytest.fixture(autouse=True)
def _fresh_states():
    from dlrover_wuqiong_amd.ops import fp8

    fp8._STATES.clear()
    fp8._DEFAULTS.clear()
    yield
    fp8._STATES.clear()
    fp8._DEFAULTS.clear()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def test_cast_records_amax_and_update_sets_scale():
    from dlrover_wuqiong_amd.ops import fp8

    st = fp8.fp8_state("cpu", history_len=4)
    i = st.register("e4m3")
    x = torch.randn(64, 32) * 3.0
    x8 = fp8.cast_to_fp8(x, st, i, "e4m3")
    assert x8.dtype == torch.float8_e4m3fn and x8.shape == x.shape
    assert st.amax_bits[i].view(torch.float32).item() == pytest.approx(x.abs().max().item())
    assert _rel(x8.float(), x) < 0.05  # scale 1: plain e4m3 rounding
    st.update()
    assert st.scale[i].item() == pytest.approx(448.0 / x.abs().max().item(), rel=1e-5)
    assert st.inv_scale[i].item() == pytest.approx(1.0 / st.scale[i].item(), rel=1e-5)
    assert st.amax_bits[i].item() == 0
    # the history keeps the max of the last 4 steps
    fp8.cast_to_fp8(x * 0.01, st, i, "e4m3")
    st.update()
    assert st.scale[i].item() == pytest.approx(448.0 / x.abs().max().item(), rel=1e-5)
    # with the new scale the values use the format's range
    x8 = fp8.cast_to_fp8(x, st, i, "e4m3")
    assert x8.float().abs().max().item() == pytest.approx(448.0, rel=0.02)
    assert _rel(x8.float() * st.inv_scale[i], x) < 0.05


def test_fp8_linear_matches_linear_forward_backward():
    from dlrover_wuqiong_amd.ops import fp8

    torch.manual_seed(0)
    ref = nn.Linear(64, 48)
    lin = nn.Linear(64, 48)
    lin.load_state_dict(ref.state_dict())
    f8 = fp8.Fp8Linear(lin, "HYBRID")
    assert f8.weight is lin.weight  # shares the parameters
    for step in range(3):
        x = torch.randn(4, 8, 64, requires_grad=True)
        xr = x.detach().clone().requires_grad_()
        y, yr = f8(x), ref(xr)
        g = torch.randn_like(yr)
        y.backward(g)
        yr.backward(g)
        assert _rel(y, yr) < 0.08, step
        assert _rel(x.grad, xr.grad) < 0.15, step
        assert _rel(lin.weight.grad, ref.weight.grad) < 0.15, step
        assert _rel(lin.bias.grad, ref.bias.grad) < 1e-5
        lin.weight.grad = lin.bias.grad = ref.weight.grad = ref.bias.grad = None
        fp8.fp8_update()  # delayed scaling advances after each step
    assert fp8.fp8_stats("cpu")["tensors"] == 3


def test_ineligible_shapes_stay_bf16():
    from dlrover_wuqiong_amd.ops import fp8

    m = nn.Sequential(nn.Linear(64, 30), nn.ReLU(), nn.Linear(30, 32), nn.Linear(32, 64))
    done = fp8.replace_linears(m, exclude=["2"])
    assert done == ["3"]  # 30 is not a multiple of 16; "2" excluded by name
    assert isinstance(m[3], fp8.Fp8Linear) and type(m[0]) is nn.Linear
    y = m[3](torch.randn(3, 32))  # 3 tokens: not a multiple of 16 -> plain GEMM
    assert y.shape == (3, 64)


def test_auto_accelerate_fp8_strategy_trains():
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
    from dlrover_wuqiong_amd.ops import fp8

    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(32, 64), nn.GELU(), nn.Linear(64, 32))
    ok, res, strategy = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": 1e-2},
                                        load_strategy=[("fp8", {"amax_history_len": 8})])
    assert ok and "fp8" in strategy.names()
    assert sum(isinstance(m, fp8.Fp8Linear) for m in res.model.modules()) == 2
    x = torch.randn(64, 32)
    target = torch.tanh(x @ torch.randn(32, 32))
    losses = []
    for _ in range(30):
        loss = (res.model(x) - target).pow(2).mean()
        loss.backward()
        res.optim.step()  # the step hook advances the FP8 scales
        res.optim.zero_grad()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0]
    st = fp8.fp8_state("cpu")
    assert st.steps == 30 and float(st.scale[: st.n].min()) != 1.0


def test_cast_nan_stays_nan_and_amax_backs_off():
    """NaN survives the saturating cast (so loss-spike / NaN checks see it),
    and the recorded amax is +inf, so the next update halves the scale --
    the contract the GPU kernels follow (tests/test_fp8_gpu.py)."""
    from dlrover_wuqiong_amd.ops import fp8

    st = fp8.fp8_state("cpu", history_len=4)
    i = st.register("e4m3")
    x = torch.randn(16, 8)
    x[2, 3] = float("nan")
    x[4, 4] = float("inf")
    x8 = fp8.cast_to_fp8(x, st, i, "e4m3").float()
    assert torch.isnan(x8[2, 3]) and x8[4, 4].item() == 448.0
    assert st.amax_bits[i].view(torch.float32).item() == float("inf")
    st.update()
    assert st.scale[i].item() == pytest.approx(0.5)


def test_fp8_with_tensor_parallel_is_rejected_loudly():
    """The verdict's silent-skip trap: fp8 under TP / SP / mixed used to be
    dropped with a warning; it now refuses."""
    import pytest

    from dlrover_wuqiong_amd.atorch.auto_accelerate import _apply_fp8

    with pytest.raises(ValueError, match="fp8 cannot be combined"):
        _apply_fp8({"tp_like": True, "model": nn.Linear(16, 16)}, None)
