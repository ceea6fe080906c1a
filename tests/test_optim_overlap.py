"""Overlapped optimizer update (optimizers/overlap.py): the forward-order
piece split of the flat buffer (CPU) -- the GPU equivalence test is
tests/test_optim_overlap_gpu.py."""

import pytest
import torch
import torch.nn as nn

from dlrover_wuqiong_amd.optimizers.overlap import forward_order_pieces
from dlrover_wuqiong_amd.parallel.flat import FlatParams


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Embedding(100, 32), *[nn.Sequential(nn.LayerNorm(32), nn.Linear(32, 32))
                                                 for _ in range(6)], nn.Linear(32, 7))


@pytest.mark.parametrize("chunks", [1, 3, 8, 100])
def test_pieces_cover_buffer_in_forward_order(chunks):
    m = _model()
    flat = FlatParams(m)
    pieces, piece_of = forward_order_pieces(flat, chunks)
    # contiguous, descending, exactly [0, numel)
    assert pieces[0][1] == flat.numel and pieces[-1][0] == 0
    for (lo, hi), (lo2, hi2) in zip(pieces, pieces[1:]):
        assert lo == hi2 and lo < hi
    assert len(pieces) <= max(1, chunks) + 1
    # every parameter lies inside its piece; forward-earlier params never in a later piece
    names = [n for n, _ in m.named_parameters()]
    order = [flat.names.index(n) for n in names]  # forward (registration) order -> flat index
    last = -1
    for i in order:
        o, c = flat.offsets[i]
        lo, hi = pieces[piece_of[i]]
        assert lo <= o and o + c <= hi
        assert piece_of[i] >= last
        last = piece_of[i]


def test_overlap_needs_gpu():
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW

    m = _model()
    opt = FusedAdamW(FlatParams(m), lr=1e-3)
    with pytest.raises(ValueError):
        opt.overlap_with_forward(m)


def test_ring_fence_taken_over_only_for_own_tensors():
    """An optimizer defers its state write-back only behind a ring snapshot
    that reads ITS tensors (a stale or foreign copier is fenced normally)."""
    import torch

    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    model = torch.nn.Linear(64, 64)
    opt = FusedAdamW(FlatParams(model), lr=1e-3)

    class Ring:
        def __init__(self, ranges):
            self.ranges = ranges

        def ring_sources(self):
            return self.ranges

    m = opt.exp_avg
    assert opt._ring_touches(Ring([(m.data_ptr(), m.data_ptr() + 16)]))
    p = opt.flat.data
    assert opt._ring_touches(Ring([(p.data_ptr() + 8, p.data_ptr() + 12)]))
    other = torch.zeros(1 << 16)
    assert not opt._ring_touches(Ring([(other.data_ptr(), other.data_ptr() + other.numel() * 4)]))
    assert not opt._ring_touches(Ring([]))
