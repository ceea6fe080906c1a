"""Compatibility import path (reference: atorch/atorch/optimizers/adam_offload.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.optimizers.offload import CPUOffloadAdamW  # noqa: F401

PartitionAdam = CPUOffloadAdamW
