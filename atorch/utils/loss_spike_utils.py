"""Compatibility import path (reference: atorch/atorch/utils/loss_spike_utils.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.utils.loss_spike import LossSpikeBase, TokenLossSpike  # noqa: F401
