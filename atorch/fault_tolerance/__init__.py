"""Compatibility import path (reference: atorch/atorch/fault_tolerance).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.fault_tolerance``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.fault_tolerance import HangingDetector, heartbeat, request_relaunch  # noqa: F401
