"""Compatibility import path (reference: dlrover/trainer/torch/flash_checkpoint/full_ckpt_engine.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.flash_checkpoint.engine``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.flash_checkpoint.engine import FullCheckpointEngine  # noqa: F401
