"""GPU: the flat AdamW kernel (optim.hip) against an
fp32 PyTorch reference of the same update -- bf16 params with fp32 master
weights, a per-64-block decay mask, ragged lengths (scalar tail) and an
offset slice (the overlapped update launches sub-ranges)."""

import pytest
import torch

from dlrover_wuqiong_amd.ops import _hip

pytestmark = pytest.mark.gpu


def _ref(w, g, m, v, mask, lr, b1, b2, eps, wd, bc1, bc2):
    decay = mask.repeat_interleave(64)[: w.numel()].bool()
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    w = torch.where(decay, w - lr * wd * w, w)
    w = w - (lr / bc1) * m / (v.sqrt() / bc2 ** 0.5 + eps)
    return w, m, v


@pytest.mark.parametrize("n,lo", [(512 * 37 + 77, 0), (1 << 20, 0), (1 << 16, 4096), (300, 0)])
def test_adam_flat_matches_fp32(n, lo):
    torch.manual_seed(0)
    dev = "cuda"
    total = lo + n
    master = torch.randn(total, device=dev)
    param = master.to(torch.bfloat16)
    grad = torch.randn(total, device=dev).to(torch.bfloat16)
    m = torch.randn(total, device=dev) * 0.1
    v = torch.rand(total, device=dev) * 0.1
    mask = (torch.rand((total + 63) // 64, device=dev) > 0.3).to(torch.uint8)
    args = dict(lr=1e-2, b1=0.9, b2=0.95, eps=1e-8, wd=0.1, bc1=1 - 0.9 ** 3, bc2=1 - 0.95 ** 3)
    wr, mr, vr = _ref(master[lo:].clone(), grad[lo:].float(), m[lo:].clone(), v[lo:].clone(), mask[lo // 64:],
                      **args)
    _hip.check(_hip.lib().dw_adam_flat(
        _hip.ptr(param[lo:]), 1, _hip.ptr(master[lo:]), _hip.ptr(grad[lo:]), 1, _hip.ptr(m[lo:]), _hip.ptr(v[lo:]),
        None, n, 0, args["lr"], args["b1"], args["b2"], args["eps"], args["wd"], args["bc1"], args["bc2"], 1,
        _hip.ptr(mask[lo // 64:]), _hip.stream()), "adam")
    torch.cuda.synchronize()
    torch.testing.assert_close(m[lo:], mr, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(v[lo:], vr, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(master[lo:], wr, rtol=1e-5, atol=1e-5)
    assert torch.equal(param[lo:], master[lo:].to(torch.bfloat16))
