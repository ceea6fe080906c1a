"""amp_native over fp32 weights on the GPU: the framework's models keep
running their bf16 HIP kernels inside the autocast region (fp32 operands are
cast at the kernel boundary, gradients reach the fp32 parameters), and the
examples' flows train (loss falls) -- vs the same model's fp32 PyTorch loss."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlrover_wuqiong_amd._native import kernels

    kernels(required=True)


@pytest.mark.parametrize("family", ["gpt2", "llama"])
def test_amp_native_fp32_model_trains_on_kernels(family):
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
    from dlrover_wuqiong_amd.ops import _hip

    torch.manual_seed(0)
    if family == "gpt2":
        from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

        cfg = GPT2Config.named("gpt2-tiny")
        model = GPT2(cfg)
    else:
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig

        cfg = LlamaConfig.named("llama-tiny")
        model = Llama(cfg)
    ref = {k: v.clone() for k, v in model.state_dict().items()}
    ok, res, _ = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": 3e-3},
                                 load_strategy=[("amp_native", {"dtype": torch.bfloat16})])
    assert ok and all(p.dtype == torch.float32 for p in res.model.parameters())
    data = torch.randint(0, cfg.vocab_size, (4, 129), device="cuda")
    # the first loss matches the fp32 model's (PyTorch math) within bf16 error
    m32 = type(model)(cfg).cuda()
    m32.load_state_dict(ref)
    with torch.no_grad():
        l32 = float(m32(data[:, :-1], data[:, 1:]))
    calls = []
    lib = _hip.lib()

    class _Count:
        def __getattr__(self, n):
            f = getattr(lib, n)
            if n.startswith("dw_") and ("norm" in n or "attn" in n):
                calls.append(n)
            return f

    orig = _hip.lib
    _hip.lib = lambda: _Count()
    try:
        losses = []
        for _ in range(15):
            loss = res.model(data[:, :-1], data[:, 1:])
            loss.backward()
            res.optim.step()
            res.optim.zero_grad()
            losses.append(float(loss))
    finally:
        _hip.lib = orig
    assert any("norm" in c for c in calls) and any("attn" in c for c in calls), set(calls)
    assert abs(losses[0] - l32) < 0.05 * abs(l32), (losses[0], l32)
    assert all(v == v for v in losses) and losses[-1] < losses[0] - 0.5, losses
    assert all(p.grad is None or p.grad.dtype == torch.float32 for p in res.model.parameters())
