"""Compatibility import path (reference: atorch/atorch/mup/shape.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.mup import (assert_hidden_size_inf, get_infshapes, get_shapes,  # noqa: F401
                                            load_base_shapes, make_base_shapes, save_base_shapes, set_base_shapes)
