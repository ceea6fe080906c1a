"""Compatibility import path (reference: atorch/atorch/optimizers/wsam.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.optimizers.wsam import WeightedSAM  # noqa: F401
