"""Compatibility import path (reference: atorch/atorch/normalization).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.ops.norm``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.ops.norm import LayerNorm, RMSNorm, layer_norm, rms_norm  # noqa: F401

AtorchLayerNorm = LayerNorm
AtorchRMSNorm = RMSNorm
