"""The LDS-DMA staging of attn_bwd_dq2.hip / attn_fwd2.hip: a
global_load_lds_dwordx4 writes LDS lane-linearly (base + 16 * lane), so each
lane fetches the global chunk that the T10(a) image (attn_common.h img_off)
places at its LDS position.  Pin, in Python, that the source-address decode
those kernels use is the exact inverse of img_off over a whole tile."""

import pytest


def img_off(D, row, ch):
    return (D * 16) * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3))


def decode(D, o):  # mirrors issue_tile() in attn_bwd_dq2.hip / attn_fwd2.hip
    rem, sub = o % (D * 16), (o % (D * 16)) % 512
    row = 8 * (o // (D * 16)) + sub // 64
    ch = 4 * (rem // 512) + (((sub % 64) // 16) ^ ((row >> 2) & 3))
    return row, ch


@pytest.mark.parametrize("D", [64, 128])
def test_lds_dma_source_decode_inverts_img_off(D):
    BK, waves = 64, 4
    tile = BK * D * 2
    seen = set()
    for piece in range(tile // 1024):
        assert piece % waves in range(waves)
        for lane in range(64):
            o = 1024 * piece + 16 * lane
            row, ch = decode(D, o)
            assert 0 <= row < BK and 0 <= ch < D // 8
            assert img_off(D, row, ch) == o
            seen.add((row, ch))
    assert len(seen) == BK * D // 8  # every 16-byte chunk of the tile exactly once
