"""Compatibility import path (reference: atorch/atorch/common/util_func.py ``data_to_device``).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.auto_accelerate``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.auto_accelerate import _default_prepare_input as data_to_device  # noqa: F401
