"""Compatibility import path (reference: dlrover/python/common).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.common``;
existing DLRover / ATorch user code imports unchanged.
"""

