"""Compatibility import path (reference: atorch/atorch/__init__.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.distributed import (init_distributed, local_rank, rank,  # noqa: F401
                                                    reset_distributed, world_size)

__version__ = "0.1.0+mi355x"


def coworker_size() -> int:
    """This framework runs no CPU co-worker processes (data preprocessing is
    done by the shm data loaders inside each rank)."""
    return 0


def __getattr__(name):
    # ``atorch.optimizers.AGD`` / ``atorch.auto`` etc. without an explicit
    # submodule import, as the reference's package allows
    import importlib

    if name in ("optimizers", "auto", "distributed", "data", "modules", "utils", "trainer", "rl", "mup", "ops",
                "local_sgd", "normalization", "fault_tolerance", "common"):
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(f"module 'atorch' has no attribute {name!r}")
