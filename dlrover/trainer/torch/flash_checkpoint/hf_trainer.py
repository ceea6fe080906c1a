"""Compatibility import path (reference: dlrover/trainer/torch/flash_checkpoint/hf_trainer.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.flash_checkpoint.hf_trainer``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.flash_checkpoint.hf_trainer import FlashCkptTrainer  # noqa: F401
