"""HuggingFace integration: run ``transformers`` models on the framework's
MFMA flash-attention kernels.

``enable_dwamd_attention(model)`` registers an attention implementation named
``"dwamd_mfma"`` with transformers' ``AttentionInterface`` and switches the
model (and every sub-config) to it, so LlamaAttention / MistralAttention /
Qwen2Attention ... call ``ops.attention.flash_attn_func`` (BSHD, GQA, causal,
head_dim 64/128) instead of SDPA; padded batches (left or right padding)
run the varlen kernels on the unpadded tokens; attention dropout and
sliding windows (Mistral / Mixtral / Qwen2 ``sliding_window``: a key is
visible iff q - W < k <= q) run on the same kernels.  Cases the kernels do
not cover -- head_dim not in {64, 128}, KV-cache decoding (q_len != k_len),
non-bf16 or CPU tensors -- fall back to transformers' own SDPA path for that
call.

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
    usable = (_hip.use_hip(query) and query.dtype == torch.bfloat16 and D in (64, 128)
              and q_len == k_len and causal)
    sw = kwargs.get("sliding_window")
    window = (int(sw) - 1, 0) if sw is not None and k_len > int(sw) else (-1, -1)
    key_valid = None
    if usable and attention_mask is not None:
        if attention_mask.dim() != 4 or attention_mask.shape[-1] != k_len:
            usable = False
        else:
            # causal + padding: the last query row of the 4-D mask lists the
            # valid keys (left or right padding); padded batches go through
            # the varlen kernels (unpad -> packed sequences -> pad)
            last = attention_mask[:, 0, -1, :]
            key_valid = last if attention_mask.dtype == torch.bool else (last == 0)
            if bool(key_valid.all()):
                key_valid = None  # a pure causal mask: the dense kernel
    if not usable:
        return sdpa_attention_forward(module, query, key, value, attention_mask, dropout=dropout, scaling=scaling,
                                      is_causal=is_causal, **kwargs)
    q, k, v = query.transpose(1, 2), key.transpose(1, 2), value.transpose(1, 2)
    if key_valid is not None:
        from ..ops.attention import flash_attn_padded_func

        return flash_attn_padded_func(q, k, v, key_valid, causal=True, softmax_scale=scaling, dropout_p=dropout,
                                      window_size=window), None
    return flash_attn_func(q, k, v, dropout_p=dropout, causal=True, softmax_scale=scaling, window_size=window), None


def register() -> str:
    global _registered
    if not _registered:
        from transformers import AttentionInterface

        AttentionInterface.register(NAME, dwamd_attention_forward)
        try:
            # without a registered mask builder transformers hands an unknown
            # implementation no mask at all (padding would be silently lost):
            # SDPA's boolean 4-D mask (None for a pure causal batch)
            from transformers import AttentionMaskInterface
            from transformers.masking_utils import sdpa_mask

            AttentionMaskInterface.register(NAME, sdpa_mask)
        except ImportError:  # pragma: no cover - older transformers build 4-D masks for any implementation
            pass
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
