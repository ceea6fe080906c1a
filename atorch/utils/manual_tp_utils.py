"""Compatibility import path (reference: atorch/atorch/utils/manual_tp_utils.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.tp_info``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.tp_info import TPInfo  # noqa: F401
