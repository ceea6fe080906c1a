"""CPU-offloaded AdamW (native host kernel) vs torch.optim.AdamW.
Parity: reference atorch/optimizers/adam_offload.py (PartitionAdam)."""

import torch


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(64, 200), torch.nn.LayerNorm(200), torch.nn.Linear(200, 10))


def test_cpu_offload_adamw_matches_torch_adamw():
    from dlrover_wuqiong_amd.optimizers.offload import CPUOffloadAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams, default_no_decay

    m1, m2 = _model(), _model()
    flat = FlatParams(m1, direct_grads=False)
    opt = CPUOffloadAdamW(flat, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1, chunk_elems=4096, threads=3)
    decay = [p for n, p in m2.named_parameters() if not default_no_decay(n, p)]
    nodecay = [p for n, p in m2.named_parameters() if default_no_decay(n, p)]
    ref = torch.optim.AdamW([{"params": decay, "weight_decay": 0.1}, {"params": nodecay, "weight_decay": 0.0}],
                            lr=1e-2, betas=(0.9, 0.95))
    x = torch.randn(32, 64)
    for _ in range(5):
        for m in (m1, m2):
            m(x).square().mean().backward()
        opt.step()
        ref.step()
        flat.zero_grad()
        ref.zero_grad()
    for p, q in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=1e-5, rtol=1e-4)
    sd = opt.state_dict()
    assert sd["step"] == 5


def test_native_cpu_adamw_bf16_grads_and_rounding():
    from dlrover_wuqiong_amd import _native

    lib = _native.runtime()
    n = 10_000 + 13  # exercise the vector body and the scalar tail
    torch.manual_seed(1)
    p = torch.randn(n)
    g = torch.randn(n).to(torch.bfloat16)
    m = torch.randn(n).abs() * 0.1
    v = torch.randn(n).abs() * 0.1
    out = torch.empty(n, dtype=torch.bfloat16)
    p0, m0, v0 = p.clone(), m.clone(), v.clone()
    lr, b1, b2, eps, wd, bc1, bc2, gs = 1e-3, 0.9, 0.999, 1e-8, 0.1, 0.5, 0.25, 0.5
    rc = lib.dw_cpu_adamw(p.data_ptr(), g.data_ptr(), 1, m.data_ptr(), v.data_ptr(), out.data_ptr(), n, lr, b1, b2,
                          eps, wd, bc1, bc2, gs, 4)
    assert rc == 0
    gf = g.float() * gs
    m_ref = b1 * m0 + (1 - b1) * gf
    v_ref = b2 * v0 + (1 - b2) * gf * gf
    p_ref = p0 * (1 - lr * wd) - (lr / bc1) * m_ref / (v_ref.sqrt() / bc2 ** 0.5 + eps)
    assert torch.allclose(m, m_ref, atol=1e-6) and torch.allclose(v, v_ref, atol=1e-6)
    assert torch.allclose(p, p_ref, atol=1e-5)
    assert torch.equal(out, p.to(torch.bfloat16))  # round-to-nearest-even like torch
    ss = lib.dw_cpu_sumsq(g.data_ptr(), 1, n)
    assert abs(ss - float(g.double().square().sum())) < 1e-6 * ss


import pytest  # noqa: E402


@pytest.mark.gpu
def test_cpu_offload_adamw_gpu_pipeline():
    """bf16 weights/grads on the GPU, fp32 state in pinned host memory:
    chunked D2H / host AdamW / H2D pipeline matches an fp32 AdamW on the
    masters (weights compared after bf16 rounding)."""
    from dlrover_wuqiong_amd.optimizers.offload import CPUOffloadAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    dev = torch.device("cuda", 0)
    m1 = _model().to(dev, torch.bfloat16)
    flat = FlatParams(m1, direct_grads=False)
    opt = CPUOffloadAdamW(flat, lr=1e-3, weight_decay=0.0, chunk_elems=2048, threads=4)
    master = opt.master.clone().requires_grad_(True)
    ref = torch.optim.AdamW([master], lr=1e-3, weight_decay=0.0)
    x = torch.randn(32, 64, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        m1(x).float().square().mean().backward()
        master.grad = flat.grad.float().cpu()
        opt.step()
        ref.step()
        flat.zero_grad()
    torch.cuda.synchronize()
    assert torch.allclose(opt.master, master.detach(), atol=1e-6)
    assert torch.equal(flat.data.cpu(), opt.master.to(torch.bfloat16))  # H2D of RNE-rounded masters
