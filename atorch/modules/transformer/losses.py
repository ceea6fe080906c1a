"""Compatibility import path (reference: atorch/atorch/modules/transformer/losses.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.ops.cross_entropy``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.ops.cross_entropy import CrossEntropyLoss, cross_entropy  # noqa: F401
