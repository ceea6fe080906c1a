"""Compatibility import path (reference: atorch/atorch/distributed).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.distributed``;
existing DLRover / ATorch user code imports unchanged.
"""

