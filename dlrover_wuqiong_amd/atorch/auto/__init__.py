"""Reference-compatible import paths (``atorch.auto``)."""

from ..auto_accelerate import auto_accelerate, model_transform  # noqa: F401
