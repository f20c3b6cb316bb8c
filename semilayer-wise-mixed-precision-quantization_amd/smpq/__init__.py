"""smpq — MI355X-native (gfx950) semilayer-wise mixed-precision quantized convolution.

Hot path: per-output-channel fake-quantized ResNet convs (kenm-28/Semilayer-Wise-Mixed-
Precision-Quantization, functions.py:9-43 + resnet.py:22-265) run as int8-MFMA implicit-GEMM
HIP kernels in libsmpq.so (C-ABI: include/smpq.h), with BN/ReLU/residual fused.
The reference's Python API is kept by the drop-in modules ``functions``, ``resnet`` and
``imagenet`` that sit next to this package.
"""
from . import ops  # noqa: F401
from .ops import get_act_limbs, set_act_limbs  # noqa: F401
from .qconv import QConv2d, stats  # noqa: F401
from .quant import channel_wise_quantizationperchan, quantize_layer_, quantize_wgt  # noqa: F401
from .checkpoint import load_checkpoint, save_checkpoint  # noqa: F401

__all__ = ["ops", "QConv2d", "stats", "quantize_wgt", "channel_wise_quantizationperchan",
           "quantize_layer_", "set_act_limbs", "get_act_limbs", "save_checkpoint", "load_checkpoint"]
