"""Compatibility import path (reference: atorch/atorch/modules/distributed_transformer).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.parallel.context_parallel``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.parallel.context_parallel import (context_parallel_attention, gather_kv_global,  # noqa: F401
                                                           zigzag_positions, zigzag_split)
