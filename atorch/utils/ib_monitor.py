"""Compatibility import path (reference: atorch/atorch/utils/ib_monitor.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.utils.net_monitor``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.utils.net_monitor import NetStat  # noqa: F401
IBStat = NetStat
