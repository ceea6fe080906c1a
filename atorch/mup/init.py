"""Compatibility import path (reference: atorch/atorch/mup/init.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.mup import (eye_, kaiming_normal_, kaiming_uniform_, normal_, ones_,  # noqa: F401
                                            trunc_normal_, uniform_, xavier_normal_, xavier_uniform_)
