"""Compatibility import path (reference: dlrover/python/common/storage.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.common.storage``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.common.storage import (CheckpointDeletionStrategy, CheckpointStorage,  # noqa: F401
                                                KeepLatestStepStrategy, KeepStepIntervalStrategy,
                                                PosixDiskStorage, PosixStorageWithDeletion,
                                                get_checkpoint_storage)
