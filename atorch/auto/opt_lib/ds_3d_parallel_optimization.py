"""Compatibility import path (reference: atorch/atorch/auto/opt_lib/ds_3d_parallel_optimization.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.tp_info``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.tp_info import DeepSpeed3DParallelConfig  # noqa: F401
