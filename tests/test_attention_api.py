"""CPU semantics of the extended attention API (the GPU kernels are checked
against the same reference in test_attention_ext_gpu.py)."""

import math

import torch
import torch.nn.functional as F

from dlrover_wuqiong_amd.ops.attention import (FlashAttnModule, attention_reference_ext, fa2_with_glm_mask,
                                               flash_attn_func, flash_attn_varlen_func, flash_attn_with_mask_bias)


def _qkv(B=2, S=48, H=2, D=16, seed=0):
    torch.manual_seed(seed)
    return (torch.randn(B, S, H, D) for _ in range(3))


def _sdpa(q, k, v, mask):
    return F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                          attn_mask=mask).transpose(1, 2)


def test_window_matches_sdpa_mask():
    q, k, v = _qkv()
    S = q.shape[1]
    i = torch.arange(S)
    d = i[None, :] - i[:, None]
    mask = (d <= 0) & (d >= -7)
    out = flash_attn_func(q, k, v, causal=True, window_size=(7, 0))
    assert torch.allclose(out, _sdpa(q, k, v, mask), atol=1e-5)


def test_glm_mask_is_causal_or_prefix():
    q, k, v = _qkv()
    S = q.shape[1]
    g = torch.tensor([10, 30], dtype=torch.int32)
    out = fa2_with_glm_mask(q, k, v, g)
    i = torch.arange(S)
    for b in range(2):
        mask = (i[None, :] <= i[:, None]) | (i[None, :] < int(g[b]))
        assert torch.allclose(out[b:b + 1], _sdpa(q[b:b + 1], k[b:b + 1], v[b:b + 1], mask), atol=1e-5)


def test_mask_bias_and_alibi():
    q, k, v = _qkv(B=1, S=20, H=2)
    mask = torch.zeros(1, 1, 1, 20)
    mask[..., 15:] = float("-inf")
    bias = torch.randn(1, 2, 20, 20)
    out = flash_attn_with_mask_bias(q, k, v, mask=mask, bias=bias)
    assert torch.allclose(out, _sdpa(q, k, v, mask + bias), atol=1e-5)
    sl = torch.tensor([0.5, 0.25])
    i = torch.arange(20)
    alibi = -sl.view(1, 2, 1, 1) * (i[None, :] - i[:, None]).abs().float()
    out = flash_attn_func(q, k, v, alibi_slopes=sl)
    assert torch.allclose(out, _sdpa(q, k, v, alibi), atol=1e-5)


def test_dropout_scaling_and_module_modes():
    q, k, v = _qkv(B=1, S=32)
    keep = torch.rand(1, 2, 32, 32) >= 0.5
    ref = attention_reference_ext(q, k, v, dropout_p=0.5, keep_mask=keep)
    p = torch.softmax(torch.einsum("bqhd,bkhd->bhqk", q, k) / math.sqrt(16), -1) * keep / 0.5
    assert torch.allclose(ref, torch.einsum("bhqk,bkhd->bqhd", p, v), atol=1e-5)
    m = FlashAttnModule(causal=True, attention_dropout=0.5)
    m.eval()
    assert torch.allclose(m(q, k, v), flash_attn_func(q, k, v, causal=True), atol=1e-6)


def test_varlen_window_alibi_cpu_and_padding_module():
    torch.manual_seed(1)
    lens = [5, 9]
    cu = torch.tensor([0, 5, 14], dtype=torch.int32)
    q, k, v = (torch.randn(14, 2, 16) for _ in range(3))
    sl = torch.tensor([0.2, 0.1])
    out = flash_attn_varlen_func(q, k, v, cu, cu, 9, 9, causal=True, window_size=(3, 0), alibi_slopes=sl)
    for b in range(2):
        a, e = int(cu[b]), int(cu[b + 1])
        r = attention_reference_ext(q[a:e][None], k[a:e][None], v[a:e][None], causal=True, window_size=(3, 0),
                                    alibi_slopes=sl)[0]
        assert torch.allclose(out[a:e], r, atol=1e-5)
    qb, kb, vb = _qkv(B=2, S=12)
    kpm = torch.ones(2, 12, dtype=torch.bool)
    kpm[0, 8:] = False
    o = FlashAttnModule(causal=True)(qb, kb, vb, key_padding_mask=kpm)
    assert torch.allclose(o[0, :8], flash_attn_func(qb[:1, :8], kb[:1, :8], vb[:1, :8], causal=True)[0], atol=1e-5)
    assert o[0, 8:].abs().max() == 0
