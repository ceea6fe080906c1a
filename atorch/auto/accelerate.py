"""Compatibility import path (reference: atorch/atorch/auto/accelerate.py:406).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.auto_accelerate``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.auto_accelerate import (AutoAccelerateResult, Strategy,  # noqa: F401
                                                        auto_accelerate, model_transform)
