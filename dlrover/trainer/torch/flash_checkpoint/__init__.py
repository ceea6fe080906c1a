"""Compatibility import path (reference: dlrover/trainer/torch/flash_checkpoint).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.flash_checkpoint``;
existing DLRover / ATorch user code imports unchanged.
"""

