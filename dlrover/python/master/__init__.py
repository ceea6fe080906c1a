"""Compatibility import path (reference: dlrover/python/master).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.master``;
existing DLRover / ATorch user code imports unchanged.
"""

