"""transformers models on the framework's attention kernels (registry
integration).  CPU: the registered function must reproduce SDPA exactly via
its fallback; GPU: the MFMA kernel path vs the eager fp32 reference."""

import pytest
import torch


def _tiny_llama():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(vocab_size=128, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64)
    torch.manual_seed(0)
    return LlamaForCausalLM(cfg)


def test_registered_attention_matches_sdpa_on_cpu():
    from dlrover_wuqiong_amd.atorch.hf_attention import NAME, enable_dwamd_attention

    m = _tiny_llama().eval()
    ids = torch.randint(0, 128, (2, 16))
    ref = m(ids).logits
    assert enable_dwamd_attention(m)
    assert m.config._attn_implementation == NAME
    out = m(ids).logits
    assert torch.allclose(out, ref, atol=1e-5)
    assert not enable_dwamd_attention(torch.nn.Linear(2, 2))


def test_auto_accelerate_module_replace_switches_hf_attention():
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
    from dlrover_wuqiong_amd.atorch.hf_attention import NAME

    ok, res, _ = auto_accelerate(_tiny_llama(), torch.optim.AdamW, optim_args={"lr": 1e-3},
                                 load_strategy=["module_replace"])
    m = res.model
    assert m.config._attn_implementation == NAME
    ids = torch.randint(0, 128, (2, 16), device=next(m.parameters()).device)  # (cuda on a GPU box)
    m(input_ids=ids, labels=ids).loss.backward()


@pytest.mark.gpu
def test_hf_llama_on_mfma_attention_gpu():
    from dlrover_wuqiong_amd.atorch.hf_attention import enable_dwamd_attention

    m = _tiny_llama().to("cuda", torch.bfloat16)
    ref = _tiny_llama().to("cuda", torch.float32)
    ref.set_attn_implementation("eager")
    ids = torch.randint(0, 128, (2, 64), device="cuda")
    enable_dwamd_attention(m)
    out = m(input_ids=ids, labels=ids)
    r = ref(input_ids=ids, labels=ids)
    assert abs(float(out.loss) - float(r.loss)) < 2e-2 * float(r.loss)
    out.loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters() if p.requires_grad)


@pytest.mark.gpu
def test_hf_llama_padded_batch_on_varlen_kernels_gpu():
    """A left-padded batch (generation-style) runs the varlen kernels and
    matches the eager fp32 model on the real tokens."""
    from dlrover_wuqiong_amd.atorch.hf_attention import enable_dwamd_attention

    m = _tiny_llama().to("cuda", torch.bfloat16)
    ref = _tiny_llama().to("cuda", torch.float32)
    ref.set_attn_implementation("eager")
    enable_dwamd_attention(m)
    ids = torch.randint(0, 128, (2, 64), device="cuda")
    am = torch.ones(2, 64, dtype=torch.long, device="cuda")
    am[0, :20] = 0  # left padding
    am[1, 50:] = 0  # right padding
    out = m(input_ids=ids, attention_mask=am).logits.float()
    r = ref(input_ids=ids, attention_mask=am).logits
    valid = am.bool()
    err = (out[valid] - r[valid]).abs().max() / r[valid].abs().max()
    assert err < 5e-2, float(err)


def test_padded_batch_routing_on_cpu(monkeypatch):
    """The padding detection -> unpad -> varlen -> pad routing, with the
    kernels replaced by the fp32 references so it runs on the CPU."""
    import dlrover_wuqiong_amd.ops._hip as hip
    import dlrover_wuqiong_amd.ops.attention as A
    from dlrover_wuqiong_amd.atorch.hf_attention import enable_dwamd_attention

    calls = []

    def varlen(q, k, v, cq, ck, mq, mk, causal, scale):
        calls.append(int(cq[-1]))
        return A.varlen_attention_reference(q, k, v, cq, ck, causal, scale)

    monkeypatch.setattr(hip, "use_hip", lambda t: True)
    monkeypatch.setattr(A._FlashAttnVarlenFn, "apply", staticmethod(varlen))
    monkeypatch.setattr(A._FlashAttnFn, "apply", staticmethod(lambda q, k, v, c, s: A.attention_reference(q, k, v, c, s)))
    m = _tiny_llama().to(torch.bfloat16)
    ref = _tiny_llama().to(torch.float32)
    ref.set_attn_implementation("eager")
    enable_dwamd_attention(m)
    ids = torch.randint(0, 128, (2, 64))
    am = torch.ones(2, 64, dtype=torch.long)
    am[0, :20] = 0
    am[1, 50:] = 0
    out = m(input_ids=ids, attention_mask=am).logits.float()
    r = ref(input_ids=ids, attention_mask=am).logits
    valid = am.bool()
    assert calls and calls[0] == int(am.sum())  # the varlen path ran on the real tokens only
    assert ((out[valid] - r[valid]).abs().max() / r[valid].abs().max()) < 3e-2
