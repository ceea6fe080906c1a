"""Compatibility import path (reference: atorch/atorch/utils/grad_scaler.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.utils.grad_scaler``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.utils.grad_scaler import BF16GradScaler, BF16ShardedGradScaler  # noqa: F401
