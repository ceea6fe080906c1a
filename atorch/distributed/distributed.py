"""Compatibility import path (reference: atorch/atorch/distributed/distributed.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.distributed``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.distributed import *  # noqa: F401,F403
from dlrover_wuqiong_amd.atorch.distributed import (create_parallel_group, destroy_parallel_group,  # noqa: F401
                                                    init_distributed, local_rank, parallel_group,
                                                    parallel_group_and_ranks, parallel_group_size,
                                                    parallel_rank, rank, reset_distributed, world_size)
