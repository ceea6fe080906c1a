"""Compatibility import path (reference: atorch/atorch/auto/engine/).

Re-exports the MI355X-native acceleration engine in ``dlrover_wuqiong_amd.atorch.engine``.
"""

from dlrover_wuqiong_amd.atorch.engine import *  # noqa: F401,F403
