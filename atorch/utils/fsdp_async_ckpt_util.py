"""Compatibility import path (reference: atorch/atorch/utils/fsdp_async_ckpt_util.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.fsdp_flat_ckpt``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.fsdp_flat_ckpt import FsdpFlatCheckpointEngine as FsdpCheckpointEngine  # noqa: F401
from dlrover_wuqiong_amd.atorch.fsdp_flat_ckpt import load_checkpoint, save_checkpoint  # noqa: F401
from dlrover_wuqiong_amd.elastic_agent.ckpt_saver import FsdpFlatCheckpointSaver as FsdpCheckpointSaver  # noqa: F401
