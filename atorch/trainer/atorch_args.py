"""Compatibility import path (reference: atorch/atorch/trainer/atorch_args.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainingArgs

AtorchArguments = AtorchTrainingArgs
