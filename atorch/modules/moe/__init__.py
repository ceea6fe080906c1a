"""Compatibility import path (reference: atorch/atorch/modules/moe).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.parallel.moe``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.parallel.moe import Experts, MoELayer, TopKGate, all_to_all_v, grouped_mlp, moe_aux_loss  # noqa: F401

TopkGate = TopKGate
