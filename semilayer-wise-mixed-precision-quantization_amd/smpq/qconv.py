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

Channels that were never quantized (bit 32 in the reference's bookkeeping: the stem, the
downsample convs, mid-search semilayers) have no integer code; they run on the same HIP kernel
with their fp32 weights in per-channel fixed point with as many int8 limbs as the activations
(16 or 24 bits), counted in ``smpq.stats["fixed_conv"]``. The 7x7/2/3 stem on <= 4 channels runs
as a 4x4 conv over space-to-depth pixels on the same kernel. Only geometries the kernel does not
cover (groups, dilation, other convs with cin % 64 != 0 or cout % 16 != 0) fall back to
``F.conv2d`` on the GPU (counted in ``stats["fp32_conv"]``).
"""
import weakref

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops

stats = {"hip_conv": 0, "fixed_conv": 0, "fp32_conv": 0, "repack": 0}
_REGISTRY = weakref.WeakSet()


def _storage_key(t):
    return (t.device.type, t.device.index, t.untyped_storage().data_ptr())


_OWNERS = {}  # storage key -> weakref of the QConv2d found last for it (verified on every hit)


def find_owner(tensor):
    """The QConv2d whose weight shares storage with ``tensor`` (None if not a QConv2d weight)."""
    key = _storage_key(tensor)
    ref = _OWNERS.get(key)
    m = ref() if ref is not None else None
    if m is not None and m.weight.device == tensor.device and _storage_key(m.weight.data) == key:
        return m
    for m in list(_REGISTRY):
        w = m.weight
        if w.device == tensor.device and _storage_key(w.data) == key:
            _OWNERS[key] = weakref.ref(m)
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
        # bumped (smpq.engine) when this conv's caches may hold weight / BN content the host keys
        # cannot see (a write through `.data` leaves `_version` unchanged)
        self._content_gen = 0
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

    def record_quant_inplace(self, channel, bit):
        """record_quant for one channel whose step the quantizer kernel already wrote into
        ``qstep[channel]`` (smpq.quant's deferred path): the bit-width as a device fill, no upload."""
        self.qbits[channel] = bit
        self._bits_host[channel] = bit
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
        return (id(w), w.data_ptr(), w._version, w.device, self._meta_gen, id(self.qstep), self.qstep.data_ptr(),
                self.qstep._version, self.qbits._version, ops.get_act_limbs(), self._content_gen)

    def hip_supported(self):
        return (self.weight.is_cuda and self.groups == 1 and self.dilation == (1, 1)
                and self.padding_mode == "zeros" and self.stride[0] == self.stride[1]
                and self.padding[0] == self.padding[1]
                and self.in_channels % 64 == 0 and self.out_channels % 16 == 0)

    def packed(self):
        """Weight operand of the HIP conv: (codes int8 [LW, cout, K], LW, offset | None,
        wscale fp32 [cout], kind), kind one of
          'exact8'  every channel quantized, exact int8 codes (LW = 1) — the hot path;
          'exact16' every channel quantized, exact codes needing 2 limbs (e.g. 257-level ties);
          'fixed'   some channels never quantized (fp32 weights, e.g. the stem, the downsample,
                    mid-search layers): those channels in per-channel fixed point with as many
                    int8 limbs as the activations (LW = max(2, L): 16 or 24 bits);
        or None when the conv's geometry is not supported by the kernel."""
        if not self.hip_supported():
            return None
        key = self._pack_key()
        if self._pack is not None and self._pack[0] == key:
            return self._pack[1]
        res = None
        w = self.weight.detach()
        with torch.no_grad():
            if self.fully_quantized() and self.in_channels % 64 == 0:
                codes, offset, wscale, status = ops.pack_weights_ex(w, self.qstep, 1)
                st = status.cpu()
                if int(st[0]) == 0 and int(st[1]) == 0:
                    has_off = bool((offset != 0).any().item())
                    res = (codes, 1, offset if has_off else None, wscale, "exact8")
            if res is None:
                step = self.qstep if (self._bits_host > 0).any() else None
                lw = max(2, ops.get_act_limbs())
                codes, _, wscale, status = ops.pack_weights_ex(w, step, lw)
                kind = "fixed" if int(status.cpu()[2]) > 0 else "exact16"
                res = (codes, lw, None, wscale, kind)
        stats["repack"] += 1
        self._pack = (key, res)
        return res

    def s2d_stem(self):
        """Is this the 7x7/2/3 stem on <= 4 channels (resnet.py:143) that runs as a 4x4 conv over
        space-to-depth pixels?"""
        return (self.weight.is_cuda and self.in_channels <= 4 and self.kernel_size == (7, 7)
                and self.stride == (2, 2) and self.padding == (3, 3) and self.groups == 1
                and self.dilation == (1, 1) and self.padding_mode == "zeros" and self.out_channels % 16 == 0)

    def packed_s2d(self):
        """Weight operand of the space-to-depth stem: (codes int8 [LW, cout, 256], wscale fp32
        [cout], kind); quantized channels as exact codes, the others in per-channel fixed point
        with LW = max(2, L) limbs (kind 'fixed' when any channel is, else 'exact16')."""
        key = self._pack_key()
        cached = getattr(self, "_s2d_pack", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        with torch.no_grad():
            quantized = (self._bits_host > 0).any()
            codes, wscale = ops.pack_weights_s2d(self.weight.detach().float(), max(2, ops.get_act_limbs()),
                                                 step=self.qstep if quantized else None)
        res = (codes, wscale, "exact16" if self.fully_quantized() else "fixed")
        stats["repack"] += 1
        self._s2d_pack = (key, res)
        return res

    # ---- forward (module path; the fused ResNet path is smpq.engine) ------------------------
    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("smpq QConv2d is MI355X-native: move the model and input to the GPU")
        if self.s2d_stem() and x.shape[1] == self.in_channels and x.shape[2] >= 2 and x.shape[3] >= 2:
            # the reference's 7x7/2/3 stem (resnet.py:143): space-to-depth planes on the conv kernel,
            # the same codes and results as the engine's stem (engine.stem_s2d_plan)
            codes, s2d_scale, kind = self.packed_s2d()
            stats["hip_conv"] += 1
            if kind == "fixed":
                stats["fixed_conv"] += 1
            self.last_path = "hip-%s-s2d" % kind
            xc = x.float().contiguous()
            amax = ops.act_absmax(xc)
            xq = ops.image_quantize_s2d(xc, amax)
            shift = self.bias.detach().float().contiguous() if self.bias is not None else \
                torch.zeros(self.out_channels, dtype=torch.float32, device=x.device)
            y = ops.tuned_stem_conv_s2d(xq, amax, codes, x.shape[2], x.shape[3], s2d_scale.contiguous(), shift,
                                        relu=False)
            return y.permute(0, 3, 1, 2)
        pk = self.packed()
        if pk is None:
            stats["fp32_conv"] += 1
            self.last_path = "fp32"
            return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
        codes, lw, offset, wscale, kind = pk
        stats["hip_conv"] += 1
        if kind == "fixed":
            stats["fixed_conv"] += 1
        self.last_path = "hip-" + kind
        x = x.float()
        xh = x.permute(0, 2, 3, 1).contiguous()
        amax = ops.act_absmax(xh)
        xq = ops.act_quantize(xh, amax)
        shift = self.bias.detach().float().contiguous() if self.bias is not None else \
            torch.zeros(self.out_channels, dtype=torch.float32, device=x.device)
        y = ops.tuned_conv2d_q(xq, amax, codes, offset, self.kernel_size[0], self.kernel_size[1],
                               self.stride[0], self.padding[0], wscale.contiguous(), shift)
        return y.permute(0, 3, 1, 2)
