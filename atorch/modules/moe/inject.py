"""Compatibility import path (reference: atorch/atorch/modules/moe/inject.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.parallel.moe``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.parallel.moe import replace_with_moe  # noqa: F401
