"""Compatibility import path (reference: atorch/atorch/optimizers/__init__.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.optimizers``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.optimizers.agd import AGD  # noqa: F401
from dlrover_wuqiong_amd.optimizers.bf16 import BF16Optimizer  # noqa: F401
from dlrover_wuqiong_amd.optimizers.low_bit import Q_CAME, Q_AGD, Q_Adafactor, Q_AdamW  # noqa: F401
from dlrover_wuqiong_amd.optimizers.offload import CPUOffloadAdamW  # noqa: F401
from dlrover_wuqiong_amd.optimizers.wsam import WeightedSAM  # noqa: F401
