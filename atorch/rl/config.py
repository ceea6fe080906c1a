"""Compatibility import path (reference: atorch/atorch/rl/config.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.rl``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.rl.rl_config import (AtorchRLConfig, GenerationConfig, ModelConfig,  # noqa: F401
                                                     OptimizerSpec as Optimizer, PPOMethodConfig as PPOConfig,
                                                     TokenizerConfig, TrainableModelConfig, TrainConfig,
                                                     is_trainable_model)

GeneratationConfig = GenerationConfig  # the reference's spelling
