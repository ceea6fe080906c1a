"""Compatibility import path (reference: atorch/atorch/rl/trainer/ppo_trainer.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.rl``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.rl.trainer import PPOTrainer  # noqa: F401
