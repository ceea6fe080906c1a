"""Compatibility import path (reference: atorch/atorch/rl/model_engine/model_engine.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.rl``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.rl.engine import ModelEngine, ValueModel  # noqa: F401
from dlrover_wuqiong_amd.atorch.rl.rl_config import build_engine  # noqa: F401
