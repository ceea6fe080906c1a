"""Compatibility import path (reference: dlrover/trainer/torch/flash_checkpoint/megatron.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.flash_checkpoint.megatron``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType  # noqa: F401
from dlrover_wuqiong_amd.flash_checkpoint.megatron import (MegatronCheckpointer, get_checkpoint_name,  # noqa: F401
                                                          load_checkpoint, save_checkpoint)
