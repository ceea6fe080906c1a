"""Compatibility import path (reference: dlrover/trainer/torch/flash_checkpoint/fsdp.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.flash_checkpoint.fsdp``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType  # noqa: F401
from dlrover_wuqiong_amd.flash_checkpoint.fsdp import FsdpFullCheckpointer, FsdpShardCheckpointer  # noqa: F401
