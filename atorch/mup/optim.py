"""Compatibility import path (reference: atorch/atorch/mup/optim.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.mup import (MuAdam, MuAdamParamGroupsAdjust, MuAdamW, MuSGD,  # noqa: F401
                                            MuSGDParamGroupsAdjust)
