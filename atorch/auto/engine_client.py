"""Compatibility import path (reference: atorch/atorch/auto/engine_client.py)."""

from dlrover_wuqiong_amd.atorch.engine.service import EngineClient  # noqa: F401
