"""Compatibility import path (reference: atorch/atorch/modules/moe/switch_gating.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.parallel.moe``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.parallel.moe import SwitchGate, capacity_mask  # noqa: F401
