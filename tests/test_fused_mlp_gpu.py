"""GPU: hipBLASLt epilogue-fused GPT MLP (bias+GELU forward, dGELU+bias-grad
backward) vs an fp32 PyTorch reference, with autograd and with flat-buffer
direct gradients."""

import pytest
import torch
import torch.nn.functional as F

from dlrover_wuqiong_amd.ops import mlp as mlp_mod

pytestmark = pytest.mark.gpu


def _ref(x, w1, b1, w2, b2):
    h = F.gelu(x.float() @ w1.float().t() + b1.float(), approximate="tanh")
    return h @ w2.float().t() + b2.float()


@pytest.mark.parametrize("mode", ["unfused", "bgrad", "dgelu"])
@pytest.mark.parametrize("M,C", [(512, 256), (1000, 1600)])
def test_fused_mlp_matches_fp32(M, C, mode, monkeypatch):
    monkeypatch.setattr(mlp_mod, "_BWD_DEFAULT", mode)
    mlp_mod._BWD_MODE.clear()
    torch.manual_seed(0)
    fc = torch.nn.Linear(C, 4 * C).cuda().to(torch.bfloat16)
    proj = torch.nn.Linear(4 * C, C).cuda().to(torch.bfloat16)
    with torch.no_grad():
        fc.bias.normal_(0, 0.5)
        proj.bias.normal_(0, 0.5)
    x = torch.randn(2, M // 2, C, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = mlp_mod.fused_gelu_mlp(x, fc, proj)
    dy = torch.randn_like(y)
    y.backward(dy)
    xs = x.detach().float().requires_grad_()
    ps = [p.detach().float().requires_grad_() for p in (fc.weight, fc.bias, proj.weight, proj.bias)]
    yr = _ref(xs, *ps)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    for got, ref in ((x.grad, xs.grad), (fc.weight.grad, ps[0].grad), (fc.bias.grad, ps[1].grad),
                     (proj.weight.grad, ps[2].grad), (proj.bias.grad, ps[3].grad)):
        scale = ref.abs().max().item()
        assert (got.float() - ref).abs().max().item() <= 3e-2 * scale + 3e-2, (got.shape, scale)
    print("backward epilogue modes:", mlp_mod._BWD_MODE)


def test_gpt2_fused_mlp_flat_grads_match_unfused(monkeypatch):
    from dlrover_wuqiong_amd.models import gpt2 as g2
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    grads = {}
    for fused in (True, False):
        monkeypatch.setattr(g2, "_FUSED_MLP", fused)
        torch.manual_seed(0)
        cfg = GPT2Config.named("gpt2-tiny") if hasattr(GPT2Config, "named") else GPT2Config()
        with torch.device("cuda"):
            m = GPT2(cfg)
        m.to(torch.bfloat16)
        flat = FlatParams(m, dtype=torch.bfloat16, device=torch.device("cuda"))
        ids = torch.randint(0, cfg.vocab_size, (2, 65), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
        loss = m(ids[:, :-1], ids[:, 1:])
        loss.backward()
        torch.cuda.synchronize()
        grads[fused] = (float(loss), flat.grad.float().clone())
    assert abs(grads[True][0] - grads[False][0]) < 1e-2
    a, b = grads[True][1], grads[False][1]
    assert (a - b).abs().max().item() <= 5e-2 * b.abs().max().item()
