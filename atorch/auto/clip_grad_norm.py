"""Compatibility import path (reference: atorch/atorch/auto/clip_grad_norm.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.utils.grad_clip import clip_grad_norm  # noqa: F401
