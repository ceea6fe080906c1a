"""Compatibility import path (reference: atorch/atorch/ops).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.ops``;
existing ATorch user code imports unchanged.
"""

