"""Compatibility import path (reference: setup.py:39-62 package "dlrover").

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd``;
existing DLRover / ATorch user code imports unchanged.
"""

