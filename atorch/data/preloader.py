"""Compatibility import path (reference: atorch/atorch/data/preloader.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.data.preloader import GpuPreLoader  # noqa: F401
