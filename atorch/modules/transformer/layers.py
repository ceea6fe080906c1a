"""Compatibility import path (reference: atorch/atorch/modules/transformer/layers.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.ops.attention``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.ops.attention import (flash_attn_func, flash_attn_padded_func,  # noqa: F401
                                               flash_attn_qkvpacked_func, flash_attn_varlen_func, pad_input,
                                               unpad_input)
