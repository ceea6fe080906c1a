"""Compatibility import path (reference: atorch/atorch/auto/engine/acceleration_engine.py)."""

from dlrover_wuqiong_amd.atorch.engine.service import AccelerationEngine  # noqa: F401
