"""Compatibility import path (reference: atorch/atorch/rl/__init__.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.rl``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.rl import *  # noqa: F401,F403
from dlrover_wuqiong_amd.atorch.rl import AtorchRLConfig, ModelEngine, PPOConfig, PPOTrainer, RLTrainer  # noqa: F401
