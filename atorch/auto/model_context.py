"""Compatibility import path (reference: atorch/atorch/auto/model_context.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.auto_accelerate``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.auto_accelerate import get_data_partition_rank_and_size  # noqa: F401
