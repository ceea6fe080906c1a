"""Compatibility import path (reference: atorch/atorch/utils/prof.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.utils.prof``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.utils.prof import AProfiler, flash_attn_flops  # noqa: F401
