"""Compatibility import path (reference: atorch/atorch/mup/module.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.mup import MupLinear, MupModule, MuReadout, MuSharedReadout, QKVLayer, QLayer  # noqa: F401

OutputLayer = MuReadout
SharedOutputLayer = MuSharedReadout
