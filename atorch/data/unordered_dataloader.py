"""Compatibility import path (reference: atorch/atorch/data/unordered_dataloader.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.data.unordered_dataloader import UnorderedDataLoader  # noqa: F401
