"""Compatibility import path (reference: atorch/atorch/normalization/layernorm.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.ops.norm import LayerNorm

AtorchLayerNorm = LayerNorm
