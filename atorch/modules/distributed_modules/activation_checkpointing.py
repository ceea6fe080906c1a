"""Compatibility import path (reference: atorch/atorch/modules/distributed_modules/activation_checkpointing.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.parallel.randomizer``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.parallel.randomizer import (CudaRNGStatesTracker, get_cuda_rng_tracker,  # noqa: F401
                                                     model_parallel_cuda_manual_seed, tp_wrap_fn)
from dlrover_wuqiong_amd.parallel.randomizer import rng_checkpoint as checkpoint  # noqa: F401
