"""Compatibility import path (reference: atorch/atorch/auto/__init__.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.auto_accelerate``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate, model_transform  # noqa: F401
