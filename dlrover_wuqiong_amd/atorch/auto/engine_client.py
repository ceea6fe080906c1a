"""``atorch.auto.engine_client`` compat path."""

from ..engine.service import EngineClient  # noqa: F401
