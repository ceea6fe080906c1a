"""Compatibility import path (reference: dlrover/trainer/torch/flash_checkpoint/engine.py:136-435).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.flash_checkpoint.engine``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.flash_checkpoint.engine import (CheckpointEngine, check_all_rank_ready,  # noqa: F401
                                                        verify_all_rank_step_consistent)
