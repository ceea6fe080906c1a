"""Compatibility import path (reference: atorch/atorch/utils/numberic_checker.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.utils.numeric_checker import NumericChecker, module_numeric_checker  # noqa: F401

module_numberic_checker = module_numeric_checker
