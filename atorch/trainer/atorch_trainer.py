"""Compatibility import path (reference: atorch/atorch/trainer/atorch_trainer.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainer  # noqa: F401
from dlrover_wuqiong_amd.atorch.utils.grad_clip import count_model_params  # noqa: F401
