"""RLHF with PPO on the framework's models and kernels (``atorch/rl``)."""

from .config import PPOConfig  # noqa: F401
from .engine import ModelEngine, ValueModel  # noqa: F401
from .trainer import PPOTrainer, RLTrainer  # noqa: F401
