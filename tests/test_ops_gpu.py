"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference (GPU)."""

import math

import pytest
import torch
import torch.nn.functional as F

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


@pytest.mark.parametrize("H,R", [(256, 777), (1000, 333), (1600, 777), (4096, 777), (8192, 777), (1600, 9000)])
@pytest.mark.parametrize("rms", [False, True])
def test_norm_fwd_bwd(H, R, rms):
    """H <= 4096: one-pass backward (dx + weight grads, row-striding waves,
    last-block finish); 8192: row pass + column-reduction pass."""
    from dlrover_wuqiong_amd.ops.norm import layer_norm, rms_norm

    torch.manual_seed(0)
    x = torch.randn(R, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_()
    dy = torch.randn(R, H, device=DEV, dtype=torch.bfloat16)
    xf, wf, bf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    if rms:
        y = rms_norm(x, w, 1e-6)
        yr = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * wf
    else:
        y = layer_norm(x, w, b, 1e-5)
        yr = F.layer_norm(xf, (H,), wf, bf, 1e-5)
    assert _rel(y, yr) < 1e-2
    y.backward(dy)
    yr.backward(dy.float())
    assert _rel(x.grad, xf.grad) < 2e-2
    assert _rel(w.grad, wf.grad) < 2e-2
    if not rms:
        assert _rel(b.grad, bf.grad) < 2e-2


@pytest.mark.parametrize("H", [256, 1600])
@pytest.mark.parametrize("rms", [False, True])
def test_add_norm_fused(H, rms):
    """(norm(x + r), x + r) with both outputs used downstream (as in the
    split residual stream) vs fp32 autograd; also exercises the self-cleaning
    workspace across repeated calls."""
    from dlrover_wuqiong_amd.ops.norm import add_layer_norm, add_rms_norm

    torch.manual_seed(1)
    for _ in range(2):
        x = torch.randn(513, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
        r = torch.randn(513, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
        w = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_()
        b = (0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_()
        dy = torch.randn(513, H, device=DEV, dtype=torch.bfloat16)
        dh = torch.randn(513, H, device=DEV, dtype=torch.bfloat16)
        xf, rf = x.detach().float().requires_grad_(), r.detach().float().requires_grad_()
        wf, bf = w.detach().float().requires_grad_(), b.detach().float().requires_grad_()
        if rms:
            y, h = add_rms_norm(x, r, w, 1e-6)
            hf = xf + rf
            yr = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-6) * wf
        else:
            y, h = add_layer_norm(x, r, w, b, 1e-5)
            hf = xf + rf
            yr = F.layer_norm(hf, (H,), wf, bf, 1e-5)
        assert _rel(h, hf) < 5e-3 and _rel(y, yr) < 1e-2
        torch.autograd.backward([y, h], [dy, dh])
        torch.autograd.backward([yr, hf], [dy.float(), dh.float()])
        assert _rel(x.grad, xf.grad) < 2e-2 and _rel(r.grad, rf.grad) < 2e-2
        assert _rel(w.grad, wf.grad) < 2e-2
        if not rms:
            assert _rel(b.grad, bf.grad) < 2e-2


def test_bias_gelu():
    from dlrover_wuqiong_amd.ops.activation import bias_gelu

    x = torch.randn(300, 6400, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(6400, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = bias_gelu(x, b)
    xf, bf = x.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = F.gelu(xf + bf, approximate="tanh")
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    assert _rel(x.grad, xf.grad) < 2e-2
    assert _rel(b.grad, bf.grad) < 2e-2


@pytest.mark.parametrize("R,C", [(8192, 6400), (1000, 1600), (37, 4800)])
def test_gelu_bwd_dbias_fused(R, C):
    """One-pass GELU backward + bias gradient (last-block finish, self-cleaning
    workspace): repeated calls, fp32 accumulate and bf16 write."""
    from dlrover_wuqiong_amd.ops import _hip

    torch.manual_seed(R)
    dy = torch.randn(R, C, device=DEV, dtype=torch.bfloat16)
    pre = torch.randn(R, C, device=DEV, dtype=torch.bfloat16)
    pf = pre.float().requires_grad_()
    F.gelu(pf, approximate="tanh").backward(dy.float())
    ref_dx, ref_db = pf.grad, pf.grad.sum(0)
    acc = torch.zeros(C, device=DEV, dtype=torch.float32)
    for it in range(3):
        dx = torch.empty_like(pre)
        ws = _hip.zeroed_workspace(C + (C + 511) // 512, DEV)
        _hip.check(_hip.lib().dw_gelu_bwd_dbias(_hip.ptr(dy), _hip.ptr(pre), _hip.ptr(dx), R, C, _hip.ptr(ws),
                                                _hip.ptr(acc), 1, 1, _hip.stream(), None), "gelu_bwd_dbias")
        assert _rel(dx, ref_dx) < 1e-2
        assert _rel(acc, (it + 1) * ref_db) < 1e-3
        assert int((ws[:C + (C + 511) // 512] != 0).sum()) == 0  # left all-zero (sums + counters)
    db16 = torch.empty(C, device=DEV, dtype=torch.bfloat16)
    _hip.check(_hip.lib().dw_gelu_bwd_dbias(_hip.ptr(dy), _hip.ptr(pre), _hip.ptr(dx), R, C, _hip.ptr(ws),
                                            _hip.ptr(db16), 0, 0, _hip.stream(), None), "gelu_bwd_dbias")
    assert _rel(db16, ref_db) < 1e-2


def test_swiglu():
    from dlrover_wuqiong_amd.ops.activation import swiglu

    x = torch.randn(257, 2 * 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = swiglu(x)
    xf = x.detach().float().requires_grad_()
    a, c = xf.chunk(2, -1)
    yr = F.silu(a) * c
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    assert _rel(x.grad, xf.grad) < 2e-2


def test_rope():
    from dlrover_wuqiong_amd.ops.rope import _rope_ref, apply_rope, rope_table

    B, S, NH, D = 2, 128, 8, 128
    cos, sin = rope_table(S, D, device=DEV)
    x = torch.randn(B, S, NH, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = apply_rope(x, cos, sin)
    xf = x.detach().float().requires_grad_()
    yr = _rope_ref(xf, cos, sin)
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    assert _rel(x.grad, xf.grad) < 2e-2


@pytest.mark.parametrize("D,nh,nkv,pos", [(128, 8, 2, False), (64, 4, 4, True)])
def test_qkv_split_rope_fused(D, nh, nkv, pos):
    """Fused split + RoPE of a packed QKV projection (dw_qkv_rope) against
    split views + the fp32 rope reference, forward and backward (the packed
    gradient written in one pass, v's gradient copied through)."""
    from dlrover_wuqiong_amd.ops.rope import _rope_ref, qkv_split_rope, rope_table

    B, S = 2, 96
    cos, sin = rope_table(S + 8, D, device=DEV)
    pid = torch.randint(0, S + 8, (B, S), device=DEV) if pos else None
    qkv = torch.randn(B, S, nh + 2 * nkv, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    q, k, v = qkv_split_rope(qkv, nh, nkv, cos, sin, pid)
    assert q.is_contiguous() and k.is_contiguous() and v.is_contiguous()
    qf = qkv.detach().float().requires_grad_()
    rq, rk, rv = qf.split([nh, nkv, nkv], dim=2)
    rq, rk = _rope_ref(rq, cos, sin, 1.0, pid), _rope_ref(rk, cos, sin, 1.0, pid)
    assert _rel(q, rq) < 1e-2 and _rel(k, rk) < 1e-2 and torch.equal(v.float(), rv)
    gq, gk, gv = torch.randn_like(q), torch.randn_like(k), torch.randn_like(v)
    (q.float() * gq.float()).sum().add((k.float() * gk.float()).sum()).add((v.float() * gv.float()).sum()).backward()
    (rq * gq.float()).sum().add((rk * gk.float()).sum()).add((rv * gv.float()).sum()).backward()
    assert _rel(qkv.grad, qf.grad) < 2e-2


def test_rope_bf16_table_and_bad_shape():
    """FSDP2 mixed precision casts the cos/sin layer inputs to bf16: the op
    upcasts them (never reads a bf16 table as fp32) and rejects short tables."""
    from dlrover_wuqiong_amd.ops._hip import HipKernelError
    from dlrover_wuqiong_amd.ops.rope import _rope_ref, apply_rope, rope_table

    B, S, NH, D = 1, 256, 4, 64
    cos, sin = rope_table(S, D, device=DEV)
    x = torch.randn(B, S, NH, D, device=DEV, dtype=torch.bfloat16)
    y = apply_rope(x, cos.bfloat16(), sin.bfloat16())
    assert _rel(y, _rope_ref(x.float(), cos.bfloat16().float(), sin.bfloat16().float())) < 1e-2
    with pytest.raises(HipKernelError):
        apply_rope(x, cos[: S // 2], sin[: S // 2])


def test_rope_pos_ids_validated_and_clamped():
    """pos_ids must be an integer tensor on the GPU; positions past the table
    clamp to its last row inside the kernel (never read past the table)."""
    from dlrover_wuqiong_amd.ops._hip import HipKernelError
    from dlrover_wuqiong_amd.ops.rope import _rope_ref, apply_rope, rope_table

    B, S, NH, D = 2, 64, 4, 64
    cos, sin = rope_table(S, D, device=DEV)
    x = torch.randn(B, S, NH, D, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, S, (B, S), device=DEV)
    assert _rel(apply_rope(x, cos, sin, pos), _rope_ref(x.float(), cos, sin, pos_ids=pos)) < 1e-2
    with pytest.raises(HipKernelError):
        apply_rope(x, cos, sin, pos.cpu())
    with pytest.raises(HipKernelError):
        apply_rope(x, cos, sin, pos.float())
    far = pos.clone()
    far[0, 0] = 10 * S
    y = apply_rope(x, cos, sin, far)
    torch.cuda.synchronize()
    far[0, 0] = S - 1
    assert _rel(y, _rope_ref(x.float(), cos, sin, pos_ids=far)) < 1e-2


@pytest.mark.parametrize("V", [50304, 1000])
def test_cross_entropy(V):
    from dlrover_wuqiong_amd.ops.cross_entropy import cross_entropy

    T = 513
    logits = (3 * torch.randn(T, V, device=DEV)).to(torch.bfloat16).requires_grad_()
    tgt = torch.randint(0, V, (T,), device=DEV)
    tgt[::7] = -100
    lf = logits.detach().float().requires_grad_()
    loss = cross_entropy(logits, tgt)
    ref = F.cross_entropy(lf, tgt, ignore_index=-100)
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1.0, abs(ref.item()))
    loss.backward()
    ref.backward()
    assert _rel(logits.grad, lf.grad) < 2e-2


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("S,H,HKV", [(256, 4, 4), (333, 8, 2)])
def test_flash_attention(D, causal, S, H, HKV):
    from dlrover_wuqiong_amd.ops.attention import attention_reference, flash_attn_func

    torch.manual_seed(1)
    B = 2
    q = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, HKV, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, HKV, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attn_func(q, k, v, causal=causal)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = attention_reference(qf, kf, vf, causal=causal)
    assert _rel(o, orf) < 2e-2
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    assert _rel(q.grad, qf.grad) < 3e-2
    assert _rel(k.grad, kf.grad) < 3e-2
    assert _rel(v.grad, vf.grad) < 3e-2


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("qscale,shift", [(12.0, 0.0), (0.05, 0.0), (1.0, -60.0)])
def test_flash_attention_score_ranges(D, causal, qscale, shift):
    """Peaked (large scores: the deferred-rescale offset moves many times),
    flat, and far-negative-shifted scores (the row offset is seeded from the
    first visible tile) against the fp32 reference, with the LSE."""
    from dlrover_wuqiong_amd.ops.attention import attention_reference, flash_attn_func

    torch.manual_seed(3)
    B, S, H = 1, 700, 4
    q = (torch.randn(B, S, H, D, device=DEV) * qscale).to(torch.bfloat16)
    k = torch.randn(B, S, H, D, device=DEV).to(torch.bfloat16)
    if shift:
        # a constant key component aligned with a constant query component
        # shifts every score of a row by the same large negative amount
        q[..., 0] = 1.0
        k[..., 0] = shift * math.sqrt(D)
    v = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    o = flash_attn_func(q, k, v, causal=causal)
    orf = attention_reference(q.float(), k.float(), v.float(), causal=causal)
    assert torch.isfinite(o.float()).all()
    assert _rel(o, orf) < 3e-2


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("H,HKV", [(4, 4), (8, 2)])
def test_flash_attention_varlen(D, causal, H, HKV):
    """Packed batch with empty, sub-tile, multi-block sequences and
    len_q != len_k (bottom-right causal) vs the fp32 per-sequence reference."""
    from dlrover_wuqiong_amd.ops.attention import flash_attn_varlen_func, varlen_attention_reference

    torch.manual_seed(3)
    lq = [37, 0, 300, 1, 513, 64]
    lk = [37, 5, 300, 40, 513, 64] if not causal else [50, 0, 300, 1, 520, 64]
    cu_q = torch.tensor([0] + list(__import__("itertools").accumulate(lq)), dtype=torch.int32, device=DEV)
    cu_k = torch.tensor([0] + list(__import__("itertools").accumulate(lk)), dtype=torch.int32, device=DEV)
    q = torch.randn(sum(lq), H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(sum(lk), HKV, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(sum(lk), HKV, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attn_varlen_func(q, k, v, cu_q, cu_k, max(lq), max(lk), causal=causal)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = varlen_attention_reference(qf, kf, vf, cu_q, cu_k, causal=causal)
    assert _rel(o, orf) < 2e-2
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    assert _rel(q.grad, qf.grad) < 3e-2
    assert _rel(k.grad, kf.grad) < 3e-2
    assert _rel(v.grad, vf.grad) < 3e-2


def test_flash_attention_padded_batch():
    """Left + right padded batch through unpad -> varlen -> pad equals dense
    attention of each sequence's valid tokens."""
    from dlrover_wuqiong_amd.ops.attention import attention_reference, flash_attn_padded_func

    torch.manual_seed(4)
    B, S, H, D = 3, 200, 4, 128
    q = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    mask = torch.zeros(B, S, dtype=torch.bool, device=DEV)
    mask[0, :150] = True   # right padding
    mask[1, 77:] = True    # left padding
    mask[2, :] = True
    o = flash_attn_padded_func(q, k, v, mask, causal=True)
    for b, (lo, hi) in enumerate([(0, 150), (77, 200), (0, 200)]):
        ref = attention_reference(q[b:b + 1, lo:hi].float(), k[b:b + 1, lo:hi].float(), v[b:b + 1, lo:hi].float(),
                                  causal=True)
        assert _rel(o[b:b + 1, lo:hi], ref) < 2e-2
        assert (lo == 0 or o[b, :lo].abs().max() == 0) and (hi == S or o[b, hi:].abs().max() == 0)


@pytest.mark.parametrize("D,causal,S", [(64, True, 1024), (64, False, 200), (128, True, 384)])
def test_flash_attention_qkvpacked(D, causal, S):
    """Packed [B, S, 3, H, D] path: strided q/k/v reads, packed dQKV writes."""
    from dlrover_wuqiong_amd.ops.attention import attention_reference, flash_attn_qkvpacked_func

    torch.manual_seed(2)
    B, H = 2, 5
    lin = torch.randn(B, S, 3 * H * D + 8, device=DEV, dtype=torch.bfloat16)
    qkv = lin[..., : 3 * H * D].view(B, S, 3, H, D).detach().requires_grad_()  # non-dense batch/row strides
    o = flash_attn_qkvpacked_func(qkv, causal=causal)
    qf = qkv.detach().float().requires_grad_()
    orf = attention_reference(qf[:, :, 0], qf[:, :, 1], qf[:, :, 2], causal=causal)
    assert _rel(o, orf) < 2e-2
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    for i in range(3):
        assert _rel(qkv.grad[:, :, i], qf.grad[:, :, i]) < 3e-2, i


@pytest.mark.parametrize("n", [1000, 1 << 20, (1 << 20) + 13])
def test_fused_adamw_matches_torch(n):
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    torch.manual_seed(0)
    m = torch.nn.Linear(n // 100 if n >= 1000 else 10, 100, bias=True).to(DEV)
    ref = torch.nn.Linear(m.in_features, 100, bias=True).to(DEV)
    ref.load_state_dict(m.state_dict())
    flat = FlatParams(m, dtype=torch.float32)
    opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.1, max_grad_norm=0.0)
    ropt = torch.optim.AdamW([{"params": [ref.weight], "weight_decay": 0.1},
                              {"params": [ref.bias], "weight_decay": 0.0}], lr=1e-2)
    for _ in range(3):
        x = torch.randn(8, m.in_features, device=DEV)
        m(x).square().sum().backward()
        ref(x).square().sum().backward()
        opt.step()
        ropt.step()
        flat.zero_grad()
        ropt.zero_grad()
    # elements whose second moment is ~eps^2 amplify last-bit differences of
    # the (independently computed) gradients: compare in aggregate + loosely
    assert _rel(m.weight, ref.weight) < 1e-5
    torch.testing.assert_close(m.weight, ref.weight, atol=5e-4, rtol=1e-3)
    torch.testing.assert_close(m.bias, ref.bias, atol=5e-4, rtol=1e-3)


def test_fused_agd_matches_reference():
    from dlrover_wuqiong_amd.optimizers.agd import AGD
    from dlrover_wuqiong_amd.optimizers.fused import FusedAGD
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    torch.manual_seed(0)
    m = torch.nn.Linear(64, 32).to(DEV)
    ref = torch.nn.Linear(64, 32).to(DEV)
    ref.load_state_dict(m.state_dict())
    flat = FlatParams(m, dtype=torch.float32, no_decay_fn=lambda n, p: False)
    opt = FusedAGD(flat, lr=1e-2, weight_decay=0.01, clip=0.5)
    ropt = AGD(ref.parameters(), lr=1e-2, weight_decay=0.01, clip=0.5)
    for _ in range(4):
        x = torch.randn(8, 64, device=DEV)
        m(x).square().sum().backward()
        ref(x).square().sum().backward()
        opt.step()
        ropt.step()
        flat.zero_grad()
        ropt.zero_grad()
    assert torch.allclose(m.weight, ref.weight, atol=1e-5, rtol=1e-4)


def test_multi_copy_kernel():
    from dlrover_wuqiong_amd.flash_checkpoint.copier import build_descs, launch_multi_copy

    src = torch.randint(0, 255, (5 << 20,), dtype=torch.uint8, device=DEV)
    dst = torch.zeros_like(src)
    pieces = [(src.data_ptr() + 3, dst.data_ptr() + 3, (3 << 20) + 5),
              (src.data_ptr() + (4 << 20), dst.data_ptr() + (4 << 20), 777),
              (src.data_ptr() + (4 << 20) + 1001, dst.data_ptr() + (4 << 20) + 1001, 64)]
    launch_multi_copy(build_descs(pieces, src.device))
    torch.cuda.synchronize()
    for s, d, n in pieces:
        so, do = s - src.data_ptr(), d - dst.data_ptr()
        assert torch.equal(src[so:so + n], dst[do:do + n])
    assert dst[:3].sum() == 0


def test_gpt2_tiny_trains():
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    with torch.device(DEV):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model)
    opt = FusedAdamW(flat, lr=3e-3)
    x = torch.randint(0, cfg.vocab_size, (4, 65), device=DEV)
    first = last = None
    for i in range(30):
        loss = model(x[:, :-1], x[:, 1:])
        loss.backward()
        opt.step()
        flat.zero_grad()
        first = first if first is not None else loss.item()
        last = loss.item()
    assert last < first - 1.0


def test_direct_flat_grads_match_autograd():
    """Fused ops accumulating straight into the flat grad buffer (addmm_ /
    colsum / norm finish kernels) == the autograd accumulation path."""
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    grads = []
    for direct in (True, False):
        torch.manual_seed(0)
        cfg = GPT2Config.named("gpt2-tiny")
        with torch.device(DEV):
            m = GPT2(cfg)
        m.to(torch.bfloat16)
        flat = FlatParams(m, direct_grads=direct)
        x = torch.randint(0, cfg.vocab_size, (2, 65), device=DEV)
        for _ in range(2):  # two micro-batches: accumulation
            m(x[:, :-1], x[:, 1:]).backward()
        grads.append(flat.grad.float().clone())
    assert _rel(grads[0], grads[1]) < 1e-2


def test_colsum_accumulate():
    from dlrover_wuqiong_amd.ops.activation import colsum

    x = torch.randn(4096, 1600, device=DEV, dtype=torch.bfloat16)
    out = torch.ones(1600, device=DEV, dtype=torch.bfloat16)
    colsum(x, out=out, accumulate=True)
    ref = x.float().sum(0) + 1
    assert _rel(out, ref) < 1e-2
    assert _rel(colsum(x, torch.float32), x.float().sum(0)) < 1e-4


@pytest.mark.parametrize("bits", [4, 8])
def test_low_bit_adamw_kernel_matches_reference(bits):
    """Fused 4/8-bit-state AdamW kernel == the PyTorch reference codec."""
    from dlrover_wuqiong_amd.optimizers.low_bit import Q_AdamW, dequant_m, _unpack4

    torch.manual_seed(0)
    n = 128 * 40 + 77
    p_gpu = torch.randn(n, device=DEV).to(torch.bfloat16).requires_grad_()
    p_ref = p_gpu.detach().clone().requires_grad_()
    og = Q_AdamW([p_gpu], lr=1e-2, q_bits=bits, threshold=1)
    orf = Q_AdamW([p_ref], lr=1e-2, q_bits=bits, threshold=1)
    for it in range(3):
        g = torch.randn(n, device=DEV).to(torch.bfloat16)
        p_gpu.grad = g.clone()
        p_ref.grad = g.clone()
        og.step()
        st = orf.state.get(p_ref) or None
        if st is None:
            orf._init_state(p_ref, orf.param_groups[0])
            orf.state[p_ref]["step"] = 0
        orf.state[p_ref]["step"] += 1
        t = orf.state[p_ref]["step"]
        b1, b2 = orf.param_groups[0]["betas"]
        with torch.no_grad():
            orf._ref_step(p_ref, orf.state[p_ref], orf.param_groups[0], 1 - b1 ** t, 1 - b2 ** t)
    assert _rel(p_gpu, p_ref) < 2e-3
    sg, sr = og.state[p_gpu], orf.state[p_ref]
    G = sg["ms"].numel()
    mg = dequant_m((_unpack4(sg["mq"]) if bits == 4 else sg["mq"]).view(G, 128), sg["ms"], bits)
    mr = dequant_m((_unpack4(sr["mq"]) if bits == 4 else sr["mq"]).view(G, 128), sr["ms"], bits)
    assert _rel(mg, mr) < 2e-2
