"""Compatibility import path (reference: dlrover/trainer/torch/flash_checkpoint/megatron_dist_ckpt.py).

Thin re-export onto the MI355X-native implementation in
``dlrover_wuqiong_amd.flash_checkpoint.megatron_dist_ckpt``; existing DLRover user code imports unchanged.
"""

from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType  # noqa: F401
from dlrover_wuqiong_amd.flash_checkpoint.megatron_dist_ckpt import (  # noqa: F401
    KeepLatestStepStrategy, KeepStepIntervalStrategy, MegatronDistCheckpointer, get_chained_optimizer_parameter_state,
    get_dist_optimizer_checkpoint_name, get_parameter_state, load_chained_optimizer_parameter_state, load_checkpoint,
    load_parameter_state_from_state_dict, save_checkpoint)
