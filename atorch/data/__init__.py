"""Compatibility import path (reference: atorch/atorch/data).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.data``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.data import *  # noqa: F401,F403
