"""Compatibility import path (reference: atorch/atorch/modules).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd``;
existing ATorch user code imports unchanged.
"""

