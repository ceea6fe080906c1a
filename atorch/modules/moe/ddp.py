"""Compatibility import path (reference: atorch/atorch/modules/moe/ddp.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.parallel.moe_ddp``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.parallel.moe_ddp import (MoEDistributedDataParallel,  # noqa: F401
                                                  MoEMixtureDistributedDataParallel, expert_data_parallel_group)
