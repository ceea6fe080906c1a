"""Linear weight + bias gradients through hipBLASLt's BGRADB epilogue
(gemm_epilogue.hip dw_gemm_wgrad_bgradb, ops/linear.py): dW accumulated in
place (beta 1) and db = column sums of dY, vs fp32 autograd."""

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd._native import kernels

    kernels(required=True)


@pytest.mark.parametrize("M,K,N", [(1024, 1600, 4800), (512, 256, 768)])
def test_wgrad_bgradb_matches_fp32(M, K, N):
    _need_gpu()
    from dlrover_wuqiong_amd.ops import linear as L
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    L._WGRAD_BGRAD = True  # opt-in path (slow on ROCm 7.2, still exact)

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = nn.Module()
    m.fc = L.FusedLinear(K, N).to(dev)
    ref_w = m.fc.weight.detach().float().clone().requires_grad_()
    ref_b = m.fc.bias.detach().float().clone().requires_grad_()
    m.to(torch.bfloat16)
    FlatParams(m)
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, requires_grad=True)
    for it in range(2):  # the second pass accumulates
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        m.fc(x).backward(dy)
        torch.nn.functional.linear(x.detach().float(), ref_w, ref_b).backward(dy.float())
    torch.cuda.synchronize()
    assert (M, K, N) not in L._BGRAD_OFF  # the epilogue path ran
    rel = lambda a, b: ((a.float() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(m.fc.weight.grad, ref_w.grad) < 2e-2
    assert rel(m.fc.bias.grad, ref_b.grad) < 2e-2
    L._WGRAD_BGRAD = False
