"""Grouped GEMM HIP kernel (NT forward, NN dgrad, TN wgrad) vs the fp32
per-expert reference, and the MoE layer on it."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd._native import kernels

    kernels(required=True)


@pytest.mark.parametrize("counts,K,N", [([0, 1, 130, 300], 256, 200), ([64, 0, 0, 500, 7], 520, 384),
                                        ([128] * 8, 1024, 1024)])
def test_grouped_linear_fwd_bwd(counts, K, N):
    from dlrover_wuqiong_amd.ops.grouped_gemm import grouped_linear, grouped_linear_reference, offsets_from_counts

    torch.manual_seed(0)
    E, T = len(counts), sum(counts)
    x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(E, N, K, device=DEV) / K ** 0.5).to(torch.bfloat16).requires_grad_()
    offs = offsets_from_counts(torch.tensor(counts, device=DEV), DEV)
    y = grouped_linear(x, w, offs)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    yr = grouped_linear_reference(xf, wf, offs)
    assert y.shape == (T, N) and _rel(y, yr) < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    assert _rel(x.grad, xf.grad) < 1e-2
    assert _rel(w.grad, wf.grad) < 1e-2
    for e, c in enumerate(counts):  # an expert with no tokens gets a zero gradient
        if c == 0:
            assert w.grad[e].abs().max() == 0


def test_moe_layer_grouped_gemm_matches_fp32():
    from dlrover_wuqiong_amd.parallel.moe import MoELayer

    torch.manual_seed(1)
    H, F, E = 256, 512, 8
    layer = MoELayer(H, F, E, top_k=2, device=DEV, dtype=torch.bfloat16)
    ref = MoELayer(H, F, E, top_k=2, device=DEV, dtype=torch.float32)
    ref.load_state_dict({k: v.float() for k, v in layer.state_dict().items()})
    x = torch.randn(4, 96, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    xf = x.detach().float().requires_grad_()
    y = layer(x)
    yr = ref(xf)  # fp32 tensors: the per-expert PyTorch loop
    assert _rel(y, yr) < 3e-2
    y.float().pow(2).mean().backward()
    yr.pow(2).mean().backward()
    assert _rel(x.grad, xf.grad) < 5e-2
    assert _rel(layer.experts.w1.grad, ref.experts.w1.grad) < 5e-2
