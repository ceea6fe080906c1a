"""MoE expert-parallel regroup kernel (csrc/kernels/moe_permute.hip): one
launch maps (source rank, expert)-ordered rows to (expert, source rank)
order and back, bit-exact against the torch index reference, forward and
backward (autograd uses the opposite direction)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd._native import kernels

    kernels(required=True)


@pytest.mark.parametrize("ep,L,H", [(8, 4, 256), (2, 16, 4096), (4, 1, 64), (8, 32, 1024)])
def test_moe_regroup_matches_reference(ep, L, H):
    from dlrover_wuqiong_amd.parallel.moe import _regroup_index, moe_regroup

    g = torch.Generator().manual_seed(ep * 100 + L)
    counts = torch.randint(0, 40, (ep, L), generator=g)
    counts[0, 0] = 0  # empty segments
    counts[-1, -1] = 0
    counts = counts.cuda()
    n = int(counts.sum())
    x = torch.randn(n, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = moe_regroup(x, counts, 0)
    dst = _regroup_index(counts, n)
    ref = torch.empty_like(x).index_copy_(0, dst, x.detach())
    assert torch.equal(y, ref)
    back = moe_regroup(y, counts, 1)
    assert torch.equal(back, x.detach())
    gy = torch.randn_like(y)
    y.backward(gy)
    assert torch.equal(x.grad, gy.index_select(0, dst))
    # grouped order: expert-major, within an expert source-rank-major
    e_of_row = torch.repeat_interleave(torch.arange(L, device="cuda").repeat_interleave(ep),
                                       counts.t().reshape(-1), output_size=n)
    assert torch.all(e_of_row[:-1] <= e_of_row[1:])
