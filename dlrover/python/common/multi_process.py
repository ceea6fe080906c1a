"""Compatibility import path (reference: dlrover/python/common/multi_process.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.common.multi_process``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.common.multi_process import SharedDict, SharedLock, SharedMemory, SharedQueue  # noqa: F401
