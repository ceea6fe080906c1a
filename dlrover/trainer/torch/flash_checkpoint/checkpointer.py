"""Compatibility import path (reference: dlrover/trainer/torch/flash_checkpoint/checkpointer.py:18-65).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.flash_checkpoint.checkpointer``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import Checkpointer, StorageType  # noqa: F401
