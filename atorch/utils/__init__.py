"""Compatibility import path (reference: atorch/atorch/utils).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.utils``;
existing DLRover / ATorch user code imports unchanged.
"""

