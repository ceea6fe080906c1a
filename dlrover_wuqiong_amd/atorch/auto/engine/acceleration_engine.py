"""``atorch.auto.engine.acceleration_engine`` compat path."""

from ...engine.service import AccelerationEngine  # noqa: F401
