"""Compatibility import path (reference: atorch/atorch/fault_tolerance/hanging_detector.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.fault_tolerance import HangingDetector  # noqa: F401
