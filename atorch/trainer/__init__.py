"""Compatibility import path (reference: atorch/atorch/trainer/__init__.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.trainer``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainer, AtorchTrainingArgs  # noqa: F401

AtorchArguments = AtorchTrainingArgs
