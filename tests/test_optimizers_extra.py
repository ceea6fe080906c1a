"""WSAM and low-bit (4/8-bit state) AdamW on CPU (reference paths);
GPU kernel parity lives in test_ops_gpu.py."""

import torch


def _problem(seed=0):
    torch.manual_seed(seed)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.Tanh(), torch.nn.Linear(64, 1))
    x = torch.randn(256, 32)
    y = (x[:, :4].sum(1, keepdim=True)).tanh()
    return model, x, y


def test_wsam_reduces_loss_and_matches_sam_when_gamma_half():
    from dlrover_wuqiong_amd.optimizers.wsam import WeightedSAM

    model, x, y = _problem()
    base = torch.optim.SGD(model.parameters(), lr=0.1)
    opt = WeightedSAM(model, base, rho=0.05, gamma=0.9)

    def closure():
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(x), y)
        loss.backward()
        return loss

    l0 = float(closure())
    for _ in range(30):
        opt.step(closure)
    assert float(closure()) < l0 * 0.7
    # coupled WSAM with gamma = 0.5 (alpha = 1) is plain SAM: step on g1
    model, x, y = _problem(1)
    ref = _problem(1)[0]
    opt = WeightedSAM(model, torch.optim.SGD(model.parameters(), lr=0.1), rho=0.05, gamma=0.5, decouple=False)

    def cl(m, o):
        def f():
            o.zero_grad()
            loss = torch.nn.functional.mse_loss(m(x), y)
            loss.backward()
            return loss
        return f

    opt.step(cl(model, opt))
    # manual SAM
    rsgd = torch.optim.SGD(ref.parameters(), lr=0.1)
    cl(ref, rsgd)()
    gn = torch.norm(torch.stack([p.grad.norm() for p in ref.parameters()]))
    with torch.no_grad():
        eps = [0.05 * p.grad / (gn + 1e-12) for p in ref.parameters()]
        for p, e in zip(ref.parameters(), eps):
            p.add_(e)
    cl(ref, rsgd)()
    with torch.no_grad():
        for p, e in zip(ref.parameters(), eps):
            p.sub_(e)
    rsgd.step()
    for a, b in zip(model.parameters(), ref.parameters()):
        assert torch.allclose(a, b, atol=1e-6)


def test_low_bit_adamw_trains_close_to_adamw():
    from dlrover_wuqiong_amd.optimizers.low_bit import Q_AdamW

    for bits in (4, 8):
        model, x, y = _problem()
        ref_model = _problem()[0]
        opt = Q_AdamW(model.parameters(), lr=1e-2, weight_decay=0.0, q_bits=bits, threshold=1000)
        ref = torch.optim.AdamW(ref_model.parameters(), lr=1e-2, weight_decay=0.0)
        for _ in range(60):
            for m, o in ((model, opt), (ref_model, ref)):
                o.zero_grad()
                torch.nn.functional.mse_loss(m(x), y).backward()
                o.step()
        lq = float(torch.nn.functional.mse_loss(model(x), y))
        lr_ = float(torch.nn.functional.mse_loss(ref_model(x), y))
        assert lq < 0.05 and lq < 3 * lr_ + 0.01, (bits, lq, lr_)
        # quantized states: 64x32 weight (2048 elems) -> 1 B/elem (8-bit) or 0.5 B (4-bit) per moment
        st = opt.state[model[0].weight]
        assert st["mq"].numel() == (2048 // 2 if bits == 4 else 2048)


def test_codec_roundtrip():
    from dlrover_wuqiong_amd.optimizers.low_bit import dequant_m, dequant_v, quant_m, quant_v

    x = torch.randn(10, 128)
    for bits in (4, 8):
        c, s = quant_m(x, bits)
        xr = dequant_m(c, s, bits)
        assert (xr - x).abs().max() <= s.max() * (0.13 if bits == 4 else 0.005)
        v = x.square()
        cv, sv = quant_v(v, bits)
        vr = dequant_v(cv, sv, bits)
        assert (vr > 0).all()  # zero-point free
        assert ((vr.sqrt() - v.sqrt()).abs() <= sv.sqrt()[:, None] * (1.0 / (16 if bits == 4 else 256))).all()


def test_bf16_optimizer_keeps_fp32_masters_and_skips_nonfinite():
    import torch

    from dlrover_wuqiong_amd.optimizers.bf16 import BF16Optimizer

    torch.manual_seed(0)
    ref = torch.nn.Linear(16, 8)
    lo = torch.nn.Linear(16, 8).to(torch.bfloat16)
    lo.load_state_dict({k: v.to(torch.bfloat16) for k, v in ref.state_dict().items()})
    ref.load_state_dict({k: v.float() for k, v in lo.state_dict().items()})
    opt = BF16Optimizer(torch.optim.SGD(lo.parameters(), lr=1e-3))
    ref_opt = torch.optim.SGD(ref.parameters(), lr=1e-3)
    for _ in range(20):
        x = torch.randn(4, 16)
        lo(x.bfloat16()).float().square().mean().backward()
        ref(x).square().mean().backward()
        # feed the reference the same (bf16-rounded) gradient
        for p, q in zip(ref.parameters(), lo.parameters()):
            p.grad.copy_(q.grad.float())
        opt.step()
        ref_opt.step()
        opt.zero_grad()
        ref_opt.zero_grad()
    # masters accumulate tiny updates that bf16 alone would round away
    masters = opt.master_groups[0]
    assert all(m.dtype == torch.float32 for m in masters)
    for m, r in zip(masters, ref.parameters()):
        assert torch.allclose(m, r, atol=1e-6)
    for p, m in zip(lo.parameters(), masters):
        assert torch.equal(p, m.to(torch.bfloat16))
    # non-finite gradient -> step skipped
    w0 = masters[0].clone()
    lo.weight.grad = torch.full_like(lo.weight, float("inf"))
    opt.step()
    assert opt.skipped_steps == 1 and torch.equal(masters[0], w0)
    sd = opt.state_dict()
    opt2 = BF16Optimizer(torch.optim.SGD(lo.parameters(), lr=1e-3))
    opt2.load_state_dict(sd)
    assert torch.equal(opt2.master_groups[0][0], masters[0])


def _toy_problem(seed=0):
    import torch

    g = torch.Generator().manual_seed(seed)
    w_true = torch.randn(64, 96, generator=g)
    x = torch.randn(256, 96, generator=g)
    return x, x @ w_true.T


def _fit(opt_cls, steps=150, **kw):
    import torch

    torch.manual_seed(0)
    x, y = _toy_problem()
    lin = torch.nn.Linear(96, 64)
    opt = opt_cls(lin.parameters(), **kw)
    first = None
    for _ in range(steps):
        loss = (lin(x) - y).square().mean()
        first = first if first is not None else float(loss.detach())
        loss.backward()
        opt.step()
        opt.zero_grad()
    return first, float((lin(x) - y).square().mean()), opt, lin


def test_q_adafactor_fp32_matches_transformers_adafactor():
    import torch
    from transformers.optimization import Adafactor

    from dlrover_wuqiong_amd.optimizers.low_bit import Q_Adafactor

    _, l_ref, _, lin_ref = _fit(Adafactor, steps=30, lr=None, relative_step=True, scale_parameter=True,
                                warmup_init=False)
    _, l_q, _, lin_q = _fit(Q_Adafactor, steps=30, q_bits=32, threshold=0)
    assert torch.allclose(lin_ref.weight, lin_q.weight, atol=1e-5), (l_ref, l_q)


def test_low_bit_optimizers_converge_with_small_state():
    from dlrover_wuqiong_amd.optimizers.agd import AGD
    from dlrover_wuqiong_amd.optimizers.low_bit import Q_AGD, Q_CAME, Q_Adafactor

    # fp32-state Q_AGD == AGD
    _, l_agd, _, lin_a = _fit(AGD, steps=20, lr=1e-2)
    _, l_qagd32, _, lin_b = _fit(Q_AGD, steps=20, lr=1e-2, q_bits=32)
    import torch

    assert torch.allclose(lin_a.weight, lin_b.weight, atol=1e-5)
    for cls, kw in ((Q_AGD, dict(lr=1e-2)), (Q_CAME, dict(lr=1e-2)), (Q_Adafactor, dict(lr=1e-2, beta1=0.9))):
        first, last, opt4, _ = _fit(cls, q_bits=4, threshold=1024, **kw)
        _, last32, opt32, _ = _fit(cls, q_bits=32, threshold=1024, **kw)
        assert last < 0.85 * first, (cls.__name__, first, last)
        assert last < 3 * last32 + 0.01 * first, (cls.__name__, last, last32)
        assert opt4.state_bytes() < 0.5 * opt32.state_bytes(), cls.__name__
