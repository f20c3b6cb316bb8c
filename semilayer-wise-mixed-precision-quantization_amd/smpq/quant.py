"""Drop-in weight quantizer API (functions.py:9-43) on the native library.

``quantize_wgt`` / ``channel_wise_quantizationperchan`` keep the reference's signatures and
bit-exact results (host C++ for CPU tensors, a HIP kernel for GPU tensors — both in
libsmpq.so), and additionally record the (bit, step) metadata on the owning QConv2d. The rounding
of functions.py:41 follows where the tensor lives, as the reference's own result does (torch
divides on the CPU and multiplies by a reciprocal on the GPU; ops.set_quant_semantics).
"""
import torch

from . import ops
from .qconv import find_owner


def quantize_wgt(tensor, bit):
    """functions.py:25-43: returns a NEW tensor = per-tensor asymmetric min/max fake-quant."""
    t = tensor.detach()
    work = t.to(torch.float32).contiguous().clone().reshape(1, -1)
    ops.quantize_channels_(work, [int(bit)])
    return work.reshape(t.shape).to(tensor.dtype)


def channel_wise_quantizationperchan(tensor, bit, i):
    """functions.py:9-23: quantize channel ``i`` of ``tensor`` IN PLACE; returns ``tensor``."""
    row = tensor[i]
    if tensor.dtype == torch.float32 and row.is_contiguous():
        step = ops.quantize_channels_(row.reshape(1, -1), [int(bit)])
    else:
        work = row.detach().to(torch.float32).contiguous().clone().reshape(1, -1)
        step = ops.quantize_channels_(work, [int(bit)])
        with torch.no_grad():
            row.copy_(work.reshape(row.shape))
    owner = find_owner(tensor)
    if owner is not None:
        owner.record_quant([int(i)], int(bit), step)
    return tensor


def quantize_layer_(conv, bits_host, semantics=None):
    """Vectorised channel_wise_quantizationperchan over a whole conv: one kernel launch.

    ``bits_host``: int array [cout], 0 = leave the channel. Per channel the result is
    identical to calling channel_wise_quantizationperchan(conv.weight.data, bit, c).
    """
    w = conv.weight.data
    w2d = w.reshape(w.shape[0], -1)
    assert w2d.data_ptr() == w.data_ptr() and w.is_contiguous()
    step = ops.quantize_channels_(w2d, bits_host, semantics=semantics)
    conv.record_quant_all(bits_host, step)
    return step
