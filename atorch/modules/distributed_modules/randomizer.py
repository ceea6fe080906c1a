"""Compatibility import path (reference: atorch/atorch/modules/distributed_modules/randomizer.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.parallel.randomizer``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.parallel.randomizer import (MultiDimParallelRandomizer, get_MDPRInstance,  # noqa: F401
                                                     get_randomizer, init_randomizer)
