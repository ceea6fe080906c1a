"""Compatibility import path (reference: atorch/atorch/utils/fsdp_save_util.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.fsdp_flat_ckpt``
(FSDP2 per-parameter dim-0 shards instead of FSDP1 flat parameters); existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.fsdp_flat_ckpt import (ShardTensorUtil, get_flat_model_param,  # noqa: F401
                                                      get_fsdp_optim_param, safetensors_dump, save_fsdp_flat_param,
                                                      save_fsdp_optim_param)
