"""Compatibility import path (reference: atorch/atorch/utils/meta_model_utils.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.utils.meta_init``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.utils.meta_init import init_empty_weights, materialize  # noqa: F401
