"""Compatibility import path (reference: atorch/atorch/local_sgd).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.local_sgd``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.local_sgd import *  # noqa: F401,F403
