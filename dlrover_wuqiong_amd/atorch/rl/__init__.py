"""RLHF with PPO on the framework's models and kernels (``atorch/rl``)."""

from .config import PPOConfig  # noqa: F401
from .engine import ModelEngine, ValueModel  # noqa: F401
from .replay_buffer import SampleReplayBuffer  # noqa: F401
from .rl_config import AtorchRLConfig, PromptDataset, build_engine, create_dataset  # noqa: F401
from .trainer import PPOTrainer, RLTrainer  # noqa: F401
