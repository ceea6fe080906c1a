"""Compatibility import path (reference: atorch/atorch/optimizers/bf16_optimizer.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.optimizers.bf16 import (BF16Optimizer, master_params_to_model_params,  # noqa: F401
                                                model_grads_to_master_grads)
