"""``atorch.auto.accelerate`` compat path."""

from ..auto_accelerate import AutoAccelerateResult, Strategy, auto_accelerate, model_transform  # noqa: F401
