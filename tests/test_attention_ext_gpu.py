"""Extended attention masks on the MFMA kernels vs an fp32 PyTorch reference
of the same op: sliding windows, GLM prefix masks, additive bias / masks,
ALiBi and dropout (the kernels' own keep mask), forward and backward, dense
and packed (varlen); ATorch FlashAttnModule / flash_attn_with_mask_bias /
fa2_with_glm_mask (reference atorch/atorch/modules/transformer/layers.py:
1167-1350)."""

import itertools

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd._native import kernels

    kernels(required=True)  # fail loudly if the HIP library is missing


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _qkv(B, S, H, HKV, D, seed=0):
    torch.manual_seed(seed)
    mk = lambda h: torch.randn(B, S, h, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)  # noqa: E731
    return mk(H), mk(HKV), mk(HKV)


def _check(o, orf, q, k, v, qf, kf, vf, tol_o=2e-2, tol_g=3e-2):
    assert torch.isfinite(o.float()).all()
    assert _rel(o, orf) < tol_o, _rel(o, orf)
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    for a, b in ((q, qf), (k, kf), (v, vf)):
        assert torch.isfinite(a.grad.float()).all()
        assert _rel(a.grad, b.grad) < tol_g, _rel(a.grad, b.grad)


CASES = [
    # name, causal, kwargs
    ("window_causal", True, dict(window_size=(100, 0))),
    ("window_bidir", False, dict(window_size=(70, 33))),
    ("window_left_only", False, dict(window_size=(-1, 17))),
    ("alibi", True, dict(alibi=True)),
    ("alibi_window", False, dict(alibi=True, window_size=(64, 64))),
    ("bias", False, dict(bias=True)),
    ("bias_causal", True, dict(bias=True)),
    ("glm", True, dict(glm=True)),
    ("dropout", False, dict(dropout_p=0.15)),
    ("dropout_causal_window", True, dict(dropout_p=0.1, window_size=(90, 0))),
]


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("name,causal,kw", CASES, ids=[c[0] for c in CASES])
def test_attention_ext_dense(D, name, causal, kw):
    from dlrover_wuqiong_amd.ops.attention import attention_reference_ext, dropout_keep_mask, flash_attn_func

    B, S, H, HKV = 2, 333, 4, 2
    q, k, v = _qkv(B, S, H, HKV, D, seed=sum(map(ord, name)))
    args = dict(causal=causal, window_size=kw.get("window_size", (-1, -1)))
    ref = dict(args)
    if kw.get("alibi"):
        sl = torch.tensor([0.5 ** (i + 1) for i in range(H)], device=DEV)
        args["alibi_slopes"] = ref["alibi_slopes"] = sl
    if kw.get("bias"):
        bias = torch.randn(B, 1, S, S, device=DEV) * 2.0
        bias[:, :, :, 5:40] = float("-inf")  # a masked band of keys
        args["attn_bias"] = ref["attn_bias"] = bias
    if kw.get("glm"):
        g = torch.tensor([50, 200], dtype=torch.int32, device=DEV)
        args["glm_mask"] = ref["glm_mask"] = g
    p = kw.get("dropout_p", 0.0)
    if p:
        seed = 1234 + D
        args.update(dropout_p=p, dropout_seed=seed)
        ref.update(dropout_p=p, keep_mask=dropout_keep_mask(B, H, S, p, seed))
        kept = ref["keep_mask"].float().mean().item()
        assert abs(kept - (1 - p)) < 0.01, kept
    o = flash_attn_func(q, k, v, **args)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = attention_reference_ext(qf, kf, vf, **ref)
    _check(o, orf, q, k, v, qf, kf, vf)


@pytest.mark.parametrize("D", [64, 128])
def test_attention_ext_lse_and_probs(D):
    """return_attn_probs gives flash-attn's (out, softmax_lse, None)."""
    from dlrover_wuqiong_amd.ops.attention import flash_attn_func

    B, S, H = 1, 200, 2
    q, k, v = _qkv(B, S, H, H, D, seed=5)
    o, lse, none = flash_attn_func(q, k, v, causal=True, window_size=(31, 0), return_attn_probs=True)
    assert none is None and lse.shape == (B, H, S)
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) / D ** 0.5
    i = torch.arange(S, device=DEV)
    vis = (i[None, :] <= i[:, None]) & (i[None, :] >= i[:, None] - 31)
    ref = torch.logsumexp(s.masked_fill(~vis, float("-inf")), dim=-1)
    assert (lse - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("D", [64, 128])
def test_attention_ext_varlen(D):
    """Packed batch: window + ALiBi per sequence; dropout on one sequence
    (its packed hash index space equals the dense B=1 mask)."""
    from dlrover_wuqiong_amd.ops.attention import attention_reference_ext, dropout_keep_mask, flash_attn_varlen_func

    torch.manual_seed(11)
    H = 4
    lens = [37, 300, 1, 129]
    cu = torch.tensor([0] + list(itertools.accumulate(lens)), dtype=torch.int32, device=DEV)
    T = sum(lens)
    q = torch.randn(T, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(T, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(T, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    sl = torch.tensor([0.3, 0.1, 0.05, 0.01], device=DEV)
    o = flash_attn_varlen_func(q, k, v, cu, cu, max(lens), max(lens), causal=True, window_size=(48, 0),
                               alibi_slopes=sl)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    outs = []
    for b in range(len(lens)):
        a, e = int(cu[b]), int(cu[b + 1])
        outs.append(attention_reference_ext(qf[a:e][None], kf[a:e][None], vf[a:e][None], causal=True,
                                            window_size=(48, 0), alibi_slopes=sl)[0])
    _check(o, torch.cat(outs), q, k, v, qf, kf, vf)

    # dropout: one packed sequence
    S = 257
    cu1 = torch.tensor([0, S], dtype=torch.int32, device=DEV)
    q1 = torch.randn(S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k1 = torch.randn(S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v1 = torch.randn(S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o1 = flash_attn_varlen_func(q1, k1, v1, cu1, cu1, S, S, dropout_p=0.2, causal=False, dropout_seed=77)
    keep = dropout_keep_mask(1, H, S, 0.2, 77)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q1, k1, v1))
    orf = attention_reference_ext(qf[None], kf[None], vf[None], dropout_p=0.2, keep_mask=keep)[0]
    _check(o1, orf, q1, k1, v1, qf, kf, vf)


def test_atorch_attention_module_variants():
    """FlashAttnModule: train-time dropout (eval: none), GLM mask, additive
    mask + bias, key padding -- each against the reference math."""
    from dlrover_wuqiong_amd.ops.attention import (FlashAttnModule, attention_reference_ext, fa2_with_glm_mask,
                                                   flash_attn_with_mask_bias)

    B, S, H, D = 2, 160, 4, 64
    q, k, v = _qkv(B, S, H, H, D, seed=21)
    m = FlashAttnModule(causal=True, attention_dropout=0.3).eval()
    o = m(q, k, v)
    assert _rel(o, attention_reference_ext(q.float(), k.float(), v.float(), causal=True)) < 2e-2
    m.train()
    o_tr = m(q, k, v)
    assert _rel(o_tr, o) > 1e-2  # dropout active in training

    g = torch.tensor([17, 90], dtype=torch.int32, device=DEV)
    assert _rel(fa2_with_glm_mask(q, k, v, g), attention_reference_ext(q.float(), k.float(), v.float(), causal=True,
                                                                       glm_mask=g)) < 2e-2
    mask = torch.zeros(B, 1, 1, S, device=DEV)
    mask[0, :, :, 100:] = float("-inf")
    bias = torch.randn(1, H, S, S, device=DEV)
    ref = attention_reference_ext(q.float(), k.float(), v.float(), attn_bias=mask + bias)
    assert _rel(flash_attn_with_mask_bias(q, k, v, mask=mask, bias=bias), ref) < 2e-2
    assert _rel(FlashAttnModule(causal=False)(q, k, v, additive_mask=mask, additive_bias=bias), ref) < 2e-2

    kpm = torch.ones(B, S, dtype=torch.bool, device=DEV)
    kpm[1, 120:] = False
    out = FlashAttnModule(causal=True)(q, k, v, key_padding_mask=kpm)
    r1 = attention_reference_ext(q[1:, :120].float(), k[1:, :120].float(), v[1:, :120].float(), causal=True)
    assert _rel(out[1:, :120], r1) < 2e-2 and out[1, 120:].abs().max().item() == 0.0
