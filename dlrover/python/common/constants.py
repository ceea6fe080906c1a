"""Compatibility import path (reference: dlrover/python/common/constants.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.common.constants``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.common.constants import *  # noqa: F401,F403
