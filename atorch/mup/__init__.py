"""Compatibility import path (reference: atorch/atorch/mup).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.mup``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.mup import (MuAdam, MuAdamParamGroupsAdjust, MupLinear, MupModule,  # noqa: F401
                                            MuReadout, MuSGD, MuSGDParamGroupsAdjust, MuSharedReadout, QKVLayer,
                                            QLayer, make_base_shapes, save_base_shapes, set_base_shapes)

OutputLayer = MuReadout
SharedOutputLayer = MuSharedReadout
