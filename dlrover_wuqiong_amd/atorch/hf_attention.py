"""HuggingFace integration: run ``transformers`` models on the framework's
MFMA flash-attention kernels.

``enable_dwamd_attention(model)`` registers an attention implementation named
``"dwamd_mfma"`` with transformers' ``AttentionInterface`` and switches the
model (and every sub-config) to it, so LlamaAttention / MistralAttention /
Qwen2Attention ... call ``ops.attention.flash_attn_func`` (BSHD, GQA, causal,
head_dim 64/128) instead of SDPA.  Cases the kernel does not cover -- a
padding mask, dropout, head_dim not in {64, 128}, non-bf16 or CPU tensors --
fall back to transformers' own SDPA path for that call.

``auto_accelerate``'s ``module_replace`` applies it to any
``PreTrainedModel`` together with the fused norm replacement.

Parity: ATorch ``atorch/modules/transformer/inject.py`` /
``layers.py`` (replace HF attention modules with FlashAttnModule) -- done
here through the transformers attention registry instead of module surgery.
"""

from typing import Optional

import torch

NAME = "dwamd_mfma"  # (names containing "flash" trigger transformers' flash-attn hub loader)
_registered = False


def dwamd_attention_forward(module, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor,
                            attention_mask: Optional[torch.Tensor], dropout: float = 0.0,
                            scaling: Optional[float] = None, is_causal: Optional[bool] = None, **kwargs):
    """transformers attention-interface signature: q/k/v [B, H, S, D];
    returns ([B, S, H, D], None)."""
    from transformers.integrations.sdpa_attention import sdpa_attention_forward

    from ..ops import _hip
    from ..ops.attention import flash_attn_func

    causal = is_causal if is_causal is not None else getattr(module, "is_causal", True)
    D = query.shape[-1]
    q_len, k_len = query.shape[2], key.shape[2]
    usable = (_hip.use_hip(query) and query.dtype == torch.bfloat16 and D in (64, 128) and dropout == 0.0
              and q_len == k_len and causal and kwargs.get("sliding_window") is None)
    if usable and attention_mask is not None:
        # a pure causal mask (no padding) is what the kernel implements
        usable = attention_mask.dim() == 4 and bool((attention_mask[:, :, -1, :] == 0).all()) \
            if attention_mask.dtype != torch.bool else bool(attention_mask[:, :, -1, :].all())
    if not usable:
        return sdpa_attention_forward(module, query, key, value, attention_mask, dropout=dropout, scaling=scaling,
                                      is_causal=is_causal, **kwargs)
    o = flash_attn_func(query.transpose(1, 2), key.transpose(1, 2), value.transpose(1, 2), causal=True,
                        softmax_scale=scaling)
    return o, None


def register() -> str:
    global _registered
    if not _registered:
        from transformers import AttentionInterface

        AttentionInterface.register(NAME, dwamd_attention_forward)
        _registered = True
    return NAME


def enable_dwamd_attention(model) -> bool:
    """Switch a transformers model to the MFMA flash-attention kernels.
    Returns False for models that are not transformers ``PreTrainedModel``s."""
    try:
        from transformers import PreTrainedModel
    except ImportError:  # pragma: no cover
        return False
    if not isinstance(model, PreTrainedModel):
        return False
    register()
    if hasattr(model, "set_attn_implementation"):
        model.set_attn_implementation(NAME)
    else:  # pragma: no cover - older transformers
        model.config._attn_implementation = NAME
    return True
