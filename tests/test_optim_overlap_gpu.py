"""Optimizer update overlapped with the next forward (optimizers/overlap.py)
on the GPU: bitwise the same training trajectory as the one-launch update,
for AdamW and AGD, with grad clipping; checkpoint snapshots taken while an
update is pending read the updated state."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd._native import kernels

    kernels(required=True)


def _run(overlap: bool, opt_name: str, steps: int = 4):
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW, FusedAGD
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    with torch.device(dev):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model)
    if opt_name == "adamw":
        opt = FusedAdamW(flat, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0)
    else:
        opt = FusedAGD(flat, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0)
    if overlap:
        ov = opt.overlap_with_forward(model, chunks=5)
        assert len(ov.pieces) >= 3
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randint(0, cfg.vocab_size, (steps, 2, 129), generator=g).to(dev)
    losses = []
    for s in range(steps):
        loss = model(x[s, :, :-1], x[s, :, 1:])
        loss.backward()
        opt.step()
        flat.zero_grad()
        losses.append(loss.detach())
    opt.join()
    flat.finalize_grads()  # (a no-op unless the gradients are zeroed lazily, parallel/flat.py)
    torch.cuda.synchronize()
    return ([float(v) for v in losses], flat.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(),
            None if opt.master is None else opt.master.clone(), float(flat.grad.abs().sum()))


@pytest.mark.parametrize("opt_name", ["adamw", "agd"])
def test_piecewise_update_bitwise_equal(opt_name):
    """The same gradients through the one-launch update and the piecewise
    side-stream update: bitwise the same parameters, masters and moments."""
    _need_gpu()
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW, FusedAGD
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    dev = torch.device("cuda:0")
    outs = []
    for overlap in (False, True):
        torch.manual_seed(0)
        with torch.device(dev):
            model = GPT2(GPT2Config.named("gpt2-tiny"))
        model.to(torch.bfloat16)
        flat = FlatParams(model)
        cls = FusedAdamW if opt_name == "adamw" else FusedAGD
        opt = cls(flat, lr=1e-3, weight_decay=0.1, max_grad_norm=1.0)
        if overlap:
            opt.overlap_with_forward(model, chunks=7)
        g = torch.Generator(device="cpu").manual_seed(3)
        for _ in range(3):
            flat.grad.copy_(torch.randn(flat.numel, generator=g).to(dev, flat.grad.dtype))
            opt.step()
            opt.join()
        torch.cuda.synchronize()
        outs.append([flat.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), opt.master])
    for ta, tb in zip(*outs):
        if ta is not None:
            assert torch.equal(ta, tb)


@pytest.mark.parametrize("opt_name", ["adamw", "agd"])
def test_overlapped_training_matches(opt_name, monkeypatch):
    """Training with the update under the next forward follows the plain
    run.  Deterministic-gradient mode (ordered column sums instead of float
    atomics, csrc/kernels/colred.hip) makes both runs' gradients
    reproducible, so the original 1e-5 tolerance holds for AdamW and AGD
    alike (AGD's m / max(sqrt(v), delta) amplifies any last-bit noise)."""
    _need_gpu()
    monkeypatch.setenv("DWAMD_DETERMINISTIC", "1")
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        a = _run(False, opt_name)
        b = _run(True, opt_name)
    finally:
        torch.use_deterministic_algorithms(False)
    assert all(abs(x - y) <= 1e-3 * abs(x) for x, y in zip(a[0], b[0])), (a[0], b[0])
    for ta, tb in zip(a[1:5], b[1:5]):
        if ta is not None:
            torch.testing.assert_close(ta.float(), tb.float(), rtol=2e-2, atol=1e-5)
    assert a[5] == 0.0 and b[5] == 0.0  # zero_grad deferred onto the side stream still zeroes


def test_snapshot_orders_after_pending_update(tmp_path):
    """A GpuCopier snapshot enqueued while the update is pending copies the
    UPDATED parameters (its copy stream waits for the update's event)."""
    _need_gpu()
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.optimizers.overlap import pending_events
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    with torch.device(dev):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model)
    opt = FusedAdamW(flat, lr=1e-2, max_grad_norm=1.0)
    opt.overlap_with_forward(model, chunks=4)
    x = torch.randint(0, cfg.vocab_size, (2, 65), device=dev)
    model(x[:, :-1], x[:, 1:]).backward()
    opt.step()
    assert pending_events(dev)
    # what a checkpoint copy stream does: wait for the pending update, then read
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    for e in pending_events(dev):
        s.wait_event(e)
    with torch.cuda.stream(s):
        snap = flat.data.clone()
    s.synchronize()
    opt.join()
    torch.cuda.synchronize()
    assert torch.equal(snap, flat.data)
