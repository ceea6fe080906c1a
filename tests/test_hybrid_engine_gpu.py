"""GPU: split-KV decode attention kernel vs an fp32 reference, and the
hybrid engine's cached / graph-replayed decode vs full forwards."""

import pytest
import torch

from dlrover_wuqiong_amd.atorch.rl.hybrid_engine import HybridEngine
from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig
from dlrover_wuqiong_amd.ops.attention import decode_attention, decode_attention_reference

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("H,HKV", [(8, 8), (32, 8), (16, 1), (4, 2)])
def test_decode_attention_kernel(D, H, HKV):
    torch.manual_seed(0)
    B, Smax = 3, 700
    q = torch.randn(B, H, D, device="cuda", dtype=torch.bfloat16)
    cache = torch.randn(2, B, Smax, HKV, D, device="cuda", dtype=torch.bfloat16)
    kc, vc = cache[0], cache[1]
    lens = torch.tensor([700, 1, 333], device="cuda", dtype=torch.int32)
    out = decode_attention(q, kc, vc, lens)
    ref = decode_attention_reference(q.float(), kc.float(), vc.float(), lens.cpu())
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


def _model():
    torch.manual_seed(0)
    cfg = LlamaConfig.named("llama-tiny")
    with torch.device("cuda"):
        m = Llama(cfg)
    return m.to(torch.bfloat16).eval()


@torch.no_grad()
def test_cached_decode_matches_full_forward():
    m = _model()
    B, P, T = 4, 9, 6
    ids = torch.randint(0, m.cfg.vocab_size, (B, P + T), device="cuda")
    eng = HybridEngine(m, B, 64, use_graph=False)
    logits = eng.prefill(ids[:, :P])
    torch.testing.assert_close(logits.float(), m(ids[:, :P])[:, -1].float(), atol=5e-2, rtol=5e-2)
    for t in range(T):
        logits = eng.decode(ids[:, P + t:P + t + 1])
        full = m(ids[:, :P + t + 1])[:, -1]
        torch.testing.assert_close(logits.float(), full.float(), atol=5e-2, rtol=5e-2)
    assert int(eng.cache.lens[0]) == P + T


@torch.no_grad()
def test_graph_replay_matches_eager_generation():
    m = _model()
    p = torch.randint(0, m.cfg.vocab_size, (4, 7), device="cuda")
    eager = HybridEngine(m, 4, 40, use_graph=False).generate(p, 12, temperature=0)
    graph_eng = HybridEngine(m, 4, 40, use_graph=True)
    graphed = graph_eng.generate(p, 12, temperature=0)
    assert graphed.tolist() == eager.tolist()
    # the cache advanced by exactly prompt + generated - 1 positions
    assert int(graph_eng.cache.lens[0]) == 7 + 12 - 1
