"""Drop-in weight quantizer API (functions.py:9-43) on the native library.

``quantize_wgt`` / ``channel_wise_quantizationperchan`` keep the reference's signatures and
bit-exact results (host C++ for CPU tensors, a HIP kernel for GPU tensors — both in
libsmpq.so), and additionally record the (bit, step) metadata on the owning QConv2d. The rounding
of functions.py:41 follows where the tensor lives, as the reference's own result does (torch
divides on the CPU and multiplies by a reciprocal on the GPU; ops.set_quant_semantics).
"""
import os

import torch

from . import _lib, ops
from .qconv import find_owner

# The unmodified search drivers call channel_wise_quantizationperchan once per CHANNEL
# (resnet50_main.py:189-197): a host sync per call for the constant-channel check, a bits upload
# and the metadata index writes cost ~140 us per call, 5.5 % of a driver step
# (profiles/r05_driver_quant_cost.json). With DEFER (default) a device weight's channel is
# quantized by one launch with no host sync: the bit-width comes from a device-resident table,
# the step is written straight into the owning conv's qstep, and a constant channel (the
# reference raises ZeroDivisionError at functions.py:40, leaving it untouched — so does the
# kernel) is recorded in a per-device flag that check_pending() reads: at the start of the next
# forward (smpq.engine.forward_fused), evaluation or checkpoint save, which raise the
# ZeroDivisionError there. SMPQ_QUANT_DEFER=0 restores the synchronous check per call.
DEFER = [os.environ.get("SMPQ_QUANT_DEFER", "1") != "0"]
# deferred calls between two checks: each has its own status word, so that check_pending can tell
# WHICH calls met a constant channel and undo exactly their metadata; a full ring is
# checked (one host sync per _RING calls)
_RING = 4096
_DEV = {}  # device -> {"bits": int8 [17] = 0..16, "status": int32 [_RING], "scratch": fp32 [1], "pending": [...]}


def _dev_state(device):
    st = _DEV.get(device)
    if st is None:
        st = _DEV[device] = {"bits": torch.arange(17, dtype=torch.int8, device=device),
                             "status": torch.zeros(_RING, dtype=torch.int32, device=device),
                             "scratch": torch.zeros(1, dtype=torch.float32, device=device), "pending": []}
    return st


def check_pending(device=None):
    """Raise ZeroDivisionError if a deferred channel_wise_quantizationperchan call (on ``device``,
    or any) met a constant channel (functions.py:40). One host sync, and only while calls are
    pending; the flags are cleared either way. The failing calls changed nothing (the kernel leaves
    a constant channel's weights and step untouched, as the reference's raise at functions.py:40
    does), and their bit-width metadata is restored here before raising, so bit_assignment,
    fully_quantized and checkpoint sidecars never report a channel that was not quantized. Calls
    made AFTER the failing one (before this check) were applied: the reference would not have
    reached them — the deferred error surfaces at the next forward, evaluation or save."""
    for dev, st in list(_DEV.items()):
        if (device is not None and dev != device) or not st["pending"]:
            continue
        pend, st["pending"] = st["pending"], []
        flags = st["status"][:len(pend)].tolist()
        if not any(flags):
            continue
        st["status"].zero_()
        bad = 0
        # newest first: a channel quantized twice in the pending window gets its oldest bit back
        for (owner, ch, prev), f in reversed(list(zip(pend, flags))):
            if f:
                bad += 1
                if owner is not None:
                    owner.record_quant_inplace(ch, prev)
        raise ZeroDivisionError("float division by zero (a constant channel in %d of the last %d "
                                "channel_wise_quantizationperchan calls, functions.py:40)" % (bad, len(pend)))


def _quantize_row_deferred(tensor, bit, i):
    """One channel of a contiguous fp32 device weight, no host sync (see DEFER)."""
    row = tensor[i]
    st = _dev_state(tensor.device)
    if len(st["pending"]) >= _RING:
        check_pending(tensor.device)
    owner = find_owner(tensor)
    if owner is not None and owner.qstep.device != tensor.device:
        owner = None
    step = owner.qstep[i:i + 1] if owner is not None else st["scratch"]
    k = len(st["pending"])
    lib = _lib.load()
    with torch.cuda.device(tensor.device):
        _lib.check(lib.smpq_quantize_channels_ex(_lib.ptr(row), 1, row.numel(), st["bits"].data_ptr() + int(bit),
                                                 _lib.ptr(step), st["status"].data_ptr() + 4 * k,
                                                 ops._qsem(None, True), _lib.stream_ptr()),
                   "smpq_quantize_channels_ex")
    st["pending"].append((owner, int(i), int(owner._bits_host[i]) if owner is not None else 0))
    if owner is not None:
        owner.record_quant_inplace(int(i), int(bit))  # qstep[i] was written by the kernel
    return tensor


def quantize_wgt(tensor, bit):
    """functions.py:25-43: returns a NEW tensor = per-tensor asymmetric min/max fake-quant."""
    t = tensor.detach()
    work = t.to(torch.float32).contiguous().clone().reshape(1, -1)
    ops.quantize_channels_(work, [int(bit)])
    return work.reshape(t.shape).to(tensor.dtype)


def channel_wise_quantizationperchan(tensor, bit, i):
    """functions.py:9-23: quantize channel ``i`` of ``tensor`` IN PLACE; returns ``tensor``."""
    if DEFER[0] and tensor.is_cuda and tensor.dtype == torch.float32 and 1 <= int(bit) <= 16 \
            and tensor[i].is_contiguous():
        return _quantize_row_deferred(tensor, bit, i)
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
