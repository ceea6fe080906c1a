"""Compatibility import path (reference: atorch/atorch/ops/quantizer).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.ops.quantization``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.ops.quantization import Quantizer, dequantize, quantize  # noqa: F401

CUDAQuantizer = Quantizer  # the reference name; HIP kernels on MI355X
