"""GPU: lazily zeroed flat gradients (parallel/flat.py) through the fused
ops -- Linear / MLP weight GEMMs with beta = 0 on the first contribution,
bias / norm reductions without accumulation, the add-norm folded bias --
equal the eagerly zeroed run over iterations with stale buffer contents and
with gradient accumulation."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(lazy, monkeypatch):
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    monkeypatch.delenv("DWAMD_LAZY_ZERO_GRAD", raising=False)
    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    with torch.device("cuda"):
        m = GPT2(cfg)
    m.to(torch.bfloat16)
    flat = FlatParams(m, dtype=torch.bfloat16, device=torch.device("cuda"), lazy_zero_grad=lazy)
    assert flat.lazy_zero == lazy
    g = torch.Generator("cuda").manual_seed(1)
    out = []
    for it in range(3):
        ids = torch.randint(0, cfg.vocab_size, (2, 65), device="cuda", generator=g)
        flat.zero_grad()
        if lazy:
            for p in flat.params:
                p.grad.fill_(7.0)  # stale contents of the open generation
        m(ids[:, :-1], ids[:, 1:]).backward()
        if it == 2:
            m(ids[:, :-1], ids[:, 1:]).backward()  # accumulation
        torch.cuda.synchronize()
        out.append(flat.grad.float().clone())
    return out


def test_lazy_zero_matches_eager_gpu(monkeypatch):
    eager = _run(False, monkeypatch)
    lazy = _run(True, monkeypatch)
    for a, b in zip(lazy, eager):
        assert (a - b).abs().max().item() <= 2e-2 * b.abs().max().item() + 1e-3
