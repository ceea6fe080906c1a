"""Compatibility import path (reference: atorch/atorch/data/shm_dataloader.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.data.shm_dataloader import (ShmDataLoader, create_shm_dataloader,  # noqa: F401
                                                          get_loader_size)

ShmDataloader = ShmDataLoader
