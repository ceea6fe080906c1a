"""Compatibility import path (reference: atorch/atorch/modules/moe/topk_gating.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.parallel.moe``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.parallel.moe import TopKGate, capacity_mask  # noqa: F401

TopkGate = TopKGate
