"""Deterministic-gradient mode (DWAMD_DETERMINISTIC=1 /
torch.use_deterministic_algorithms(True)): the column reductions (bias,
LayerNorm / RMSNorm weight gradients, the GELU-bias backward) combine
per-block partials in a fixed order instead of with float atomics, so two
identical runs give bit-identical gradients.  Checked against fp32 PyTorch
references too (the deterministic path is a different kernel path)."""

import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture
def det(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd._native import kernels

    kernels(required=True)
    monkeypatch.setenv("DWAMD_DETERMINISTIC", "1")
    yield


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.mark.parametrize("R,C", [(8192, 1600), (8192, 6400), (1000, 776)])
def test_colsum_and_gelu_dbias_bitwise(det, R, C):
    from dlrover_wuqiong_amd.ops import _hip
    from dlrover_wuqiong_amd.ops.activation import colsum

    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(R, C, device=DEV, dtype=torch.bfloat16, generator=g)
    outs = [colsum(x, torch.float32) for _ in range(3)]
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    assert _rel(outs[0], x.float().sum(0)) < 1e-5
    pre = torch.randn(R, C, device=DEV, dtype=torch.bfloat16, generator=g)
    res = []
    for _ in range(3):
        dx = torch.empty_like(pre)
        db = torch.empty(C, device=DEV, dtype=torch.float32)
        ws = _hip.zeroed_workspace(C + (C + 511) // 512, DEV)
        _hip.check(_hip.lib().dw_gelu_bwd_dbias(_hip.ptr(x), _hip.ptr(pre), _hip.ptr(dx), R, C, _hip.ptr(ws),
                                                _hip.ptr(db), 1, 0, _hip.stream(), _hip.det_scratch(R, C, 1, DEV)),
                   "gelu_bwd_dbias")
        res.append(db)
        assert int((ws[:C + (C + 511) // 512] != 0).sum()) == 0  # counters still self-cleaning
    assert all(torch.equal(res[0], r) for r in res[1:])
    pf = pre.float().requires_grad_()
    F.gelu(pf, approximate="tanh").backward(x.float())
    assert _rel(res[0], pf.grad.sum(0)) < 1e-3


@pytest.mark.parametrize("H,rms", [(1600, False), (4096, True), (4096, False), (1024, True)])
def test_norm_weight_grads_bitwise(det, H, rms):
    from dlrover_wuqiong_amd.ops.norm import layer_norm, rms_norm

    R = 8192
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(R, H, device=DEV, dtype=torch.bfloat16, generator=g)
    dy = torch.randn(R, H, device=DEV, dtype=torch.bfloat16, generator=g)
    w0 = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(torch.bfloat16)
    b0 = (0.1 * torch.randn(H, device=DEV, generator=g)).to(torch.bfloat16)
    grads = []
    for _ in range(3):
        w = w0.clone().requires_grad_()
        b = b0.clone().requires_grad_()
        xi = x.clone().requires_grad_()
        y = rms_norm(xi, w, 1e-5) if rms else layer_norm(xi, w, b, 1e-5)
        y.backward(dy)
        grads.append((xi.grad.clone(), w.grad.clone(), None if rms else b.grad.clone()))
    for gi in grads[1:]:
        for a, bb in zip(grads[0], gi):
            if a is not None:
                assert torch.equal(a, bb)
    xf = x.float().requires_grad_()
    wf = w0.float().requires_grad_()
    bf = b0.float().requires_grad_()
    if rms:
        yf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    else:
        yf = F.layer_norm(xf, (H,), wf, bf, 1e-5)
    yf.backward(dy.float())
    assert _rel(grads[0][1], wf.grad) < 1e-2  # bf16 weight gradients
    if not rms:
        assert _rel(grads[0][2], bf.grad) < 1e-2


def _train(steps=3):
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAGD
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    with torch.device(DEV):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model)
    opt = FusedAGD(flat, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randint(0, cfg.vocab_size, (steps, 4, 257), generator=g).to(DEV)
    grads = []
    for s in range(steps):
        model(x[s, :, :-1], x[s, :, 1:]).backward()
        grads.append(flat.grad.clone())
        opt.step()
        flat.zero_grad()
    torch.cuda.synchronize()
    return grads, flat.data.clone(), opt.exp_avg_sq.clone()


def test_two_training_runs_bitwise_identical(det):
    """The whole GPT-2 backward (embedding, attention, MLP, norms, biases) and
    the AGD update: identical flat gradients and parameters run to run."""
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        a = _train()
        b = _train()
    finally:
        torch.use_deterministic_algorithms(False)
    for ga, gb in zip(a[0], b[0]):
        assert torch.equal(ga, gb)
    assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
