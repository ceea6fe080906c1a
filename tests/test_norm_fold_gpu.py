"""Bias gradient of a Linear folded into the following add-norm's backward
(ops/norm.py _fold_target, colred.hip norm_bwd_part_kernel DS): the fused
column sums equal the fp32 autograd reference, and the Linear's own
reduction is skipped (no double counting)."""

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd._native import kernels

    kernels(required=True)


class _Blk(nn.Module):
    def __init__(self, H, rms):
        super().__init__()
        from dlrover_wuqiong_amd.ops.linear import FusedLinear
        from dlrover_wuqiong_amd.ops.norm import LayerNorm, RMSNorm

        self.proj = FusedLinear(H, H)
        self.ln = RMSNorm(H) if rms else LayerNorm(H)

    def forward(self, x, a):
        y, h = self.ln.add_forward(x, self.proj(a))
        return y, h


@pytest.mark.parametrize("H,R", [(1600, 1000), (512, 4096), (1000, 77)])
@pytest.mark.parametrize("rms", [False, True])
def test_bias_grad_folded_into_add_norm(H, R, rms):
    _need_gpu()
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = _Blk(H, rms).to(dev)
    with torch.no_grad():
        m.proj.bias.normal_(0, 0.1)
        m.ln.weight.normal_(1, 0.1)
    ref = _Blk(H, rms).to(dev).float()
    ref.load_state_dict({k: v.float() for k, v in m.state_dict().items()})
    m.to(torch.bfloat16)
    flat = FlatParams(m)  # direct flat gradients: the fold applies
    x = torch.randn(R, H, device=dev, dtype=torch.bfloat16)
    a = torch.randn(R, H, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(R, H, device=dev, dtype=torch.bfloat16)
    dh = torch.randn(R, H, device=dev, dtype=torch.bfloat16)
    for _ in range(2):  # accumulation over two backward passes
        y, h = m(x, a)
        assert getattr(h.grad_fn, "fold", None) is not None or getattr(y.grad_fn, "fold", None) is not None
        node = y.grad_fn.fold[0]
        torch.autograd.backward([y, h], [dy, dh])
        assert node.out_bias_folded
        ry, rh = ref(x.float(), a.float())
        torch.autograd.backward([ry, rh], [dy.float(), dh.float()])
    torch.cuda.synchronize()
    g = m.proj.bias.grad.float()
    gr = ref.proj.bias.grad
    assert ((g - gr).norm() / gr.norm()).item() < 2e-2
    gw = m.proj.weight.grad.float()
    assert ((gw - ref.proj.weight.grad).norm() / ref.proj.weight.grad.norm()).item() < 2e-2
    assert ((m.ln.weight.grad.float() - ref.ln.weight.grad).norm() / ref.ln.weight.grad.norm()).item() < 2e-2
