"""QConv2d: the reference's nn.Conv2d (resnet.py:22-30) carrying per-output-channel quantization
metadata so that its forward can run on the int8-MFMA HIP kernel.

The reference never records bit-widths: ``functions.channel_wise_quantizationperchan``
(functions.py:9-23) just overwrites ``conv.weight.data[i]`` with ``fl32(m * step)``. Here the
drop-in ``functions.channel_wise_quantizationperchan`` finds the QConv2d owning the tensor
(by storage) and records ``(bit, step)`` for channel ``i`` in two persistent buffers
(``qbits`` int8, ``qstep`` fp32), so they follow ``.to(device)``, ``state_dict()`` /
``torch.save`` / ``load_state_dict`` (resnet50_main.py:212,233-234,426-427) together with the
weight. The packed int8 codes are rebuilt whenever the weight or the metadata changes
(data_ptr, ``_version``, or the metadata generation), and verified bitwise against the weight
(smpq_pack_weights): a channel whose weight is not ``fl32(m * step)`` is never run through
the integer path.

Channels that were never quantized (bit 32 in the reference's bookkeeping, e.g. mid-search
semilayers) have no integer representation; a conv with any such channel runs the plain fp32
``F.conv2d`` (MIOpen) — exactly the reference's arithmetic for unquantized weights — and is
counted in ``smpq.stats``.
"""
import weakref

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops

stats = {"hip_conv": 0, "fp32_conv": 0, "repack": 0}
_REGISTRY = weakref.WeakSet()


def _storage_key(t):
    return (t.device.type, t.device.index, t.untyped_storage().data_ptr())


def find_owner(tensor):
    """The QConv2d whose weight shares storage with ``tensor`` (None if not a QConv2d weight)."""
    key = _storage_key(tensor)
    for m in list(_REGISTRY):
        w = m.weight
        if w.device == tensor.device and _storage_key(w.data) == key:
            return m
    return None


class QConv2d(nn.Conv2d):
    """nn.Conv2d + per-channel fake-quant metadata; forward on the HIP int8 path when possible."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.register_buffer("qbits", torch.zeros(self.out_channels, dtype=torch.int8))
        self.register_buffer("qstep", torch.zeros(self.out_channels, dtype=torch.float32))
        self._bits_host = np.zeros(self.out_channels, dtype=np.int16)
        self._meta_gen = 0
        self._pack = None
        self.last_path = None
        _REGISTRY.add(self)

    # ---- metadata -----------------------------------------------------------------------
    def record_quant(self, channels, bit, step):
        """Record that ``channels`` were quantized at ``bit`` with fp32 ``step`` (tensor)."""
        idx = torch.as_tensor(channels, dtype=torch.long).reshape(-1)
        self.qbits[idx.to(self.qbits.device)] = int(bit)
        self.qstep[idx.to(self.qstep.device)] = step.reshape(-1).to(self.qstep.device)
        self._bits_host[idx.numpy()] = int(bit)
        self._meta_gen += 1

    def record_quant_all(self, bits_host, step):
        """Vectorised record for a whole layer: bits_host int array [cout] (0 = untouched)."""
        bits_host = np.asarray(bits_host)
        sel = np.nonzero(bits_host > 0)[0]
        if len(sel) == 0:
            return
        idx = torch.from_numpy(sel).to(self.qbits.device)
        self.qbits[idx] = torch.from_numpy(bits_host[sel].astype(np.int8)).to(self.qbits.device)
        self.qstep[idx] = step.reshape(-1)[idx.to(step.device)].to(self.qstep.device)
        self._bits_host[sel] = bits_host[sel]
        self._meta_gen += 1

    def clear_quant(self):
        self.qbits.zero_()
        self.qstep.zero_()
        self._bits_host[:] = 0
        self._meta_gen += 1

    def fully_quantized(self):
        return bool((self._bits_host > 0).all())

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        has_meta = (prefix + "qbits") in state_dict and (prefix + "qstep") in state_dict
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)
        if has_meta:
            self._bits_host = self.qbits.detach().cpu().numpy().astype(np.int16)
        else:
            # e.g. a torchvision checkpoint (resnet.py:228-231): plain fp32 weights, no metadata
            for k in (prefix + "qbits", prefix + "qstep"):
                if k in missing_keys:
                    missing_keys.remove(k)
            with torch.no_grad():
                self.qbits.zero_()
                self.qstep.zero_()
            self._bits_host = np.zeros(self.out_channels, dtype=np.int16)
        self._meta_gen += 1

    # ---- packing ---------------------------------------------------------------------------
    def _pack_key(self):
        w = self.weight
        return (w.data_ptr(), w._version, w.device, self._meta_gen, self.qstep.data_ptr(),
                self.qstep._version, self.qbits._version)

    def packed(self):
        """(codes, offset_or_None) for the HIP kernel, or None if the layer must run in fp32."""
        if not self.weight.is_cuda or self.groups != 1 or self.dilation != (1, 1) \
                or self.in_channels % 64 != 0 or self.padding_mode != "zeros" \
                or not self.fully_quantized():
            return None
        key = self._pack_key()
        if self._pack is not None and self._pack[0] == key:
            return self._pack[1]
        with torch.no_grad():
            codes, offset, status = ops.pack_weights(self.weight.detach(), self.qstep)
            st = status.cpu()
            has_off = bool((offset != 0).any().item())
        stats["repack"] += 1
        if int(st[0]) or int(st[1]):
            res = None  # weights not on the recorded grid, or > 256 levels: fp32 path
        else:
            res = (codes, offset if has_off else None)
        self._pack = (key, res)
        return res

    # ---- forward (module path; the fused ResNet path is smpq.engine) ------------------------
    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("smpq QConv2d is MI355X-native: move the model and input to the GPU")
        pk = self.packed()
        if pk is None:
            stats["fp32_conv"] += 1
            self.last_path = "fp32"
            return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
        codes, offset = pk
        stats["hip_conv"] += 1
        self.last_path = "hip"
        xh = x.float().permute(0, 2, 3, 1).contiguous()
        amax = ops.act_absmax(xh)
        shift = self.bias.detach().float().contiguous() if self.bias is not None else \
            torch.zeros(self.out_channels, dtype=torch.float32, device=x.device)
        y = ops.conv2d_nhwc(xh, amax, codes, offset, self.kernel_size[0], self.kernel_size[1],
                            self.stride[0], self.padding[0], self.qstep.contiguous(), shift)
        return y.permute(0, 3, 1, 2)
