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
    ids = torch.randint(0, 128, (2, 16))
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
