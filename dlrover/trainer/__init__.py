"""Compatibility import path (reference: dlrover/trainer).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.trainer``;
existing DLRover / ATorch user code imports unchanged.
"""

