"""Compatibility import path (reference: dlrover/python).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd``;
existing DLRover / ATorch user code imports unchanged.
"""

