"""Tensor-level wrappers over the libsmpq C-ABI (include/smpq.h).

Every function validates shapes/dtypes/devices on the host before launching, so a kernel
never sees an operand that disagrees with its grid (no device-side faults on bad input).
"""
import os

import torch

from . import _lib

# activation code width in int8 limbs (1 = int8, 2 = int16, 3 = int24); see DESIGN.md
# Activation code width in int8 limbs: 3 (int24, the default) is the parity mode — logits within
# 2e-4 relative of the fp32 reference and identical top-1 labels; 2 (int16) is the fast mode
# (~1e-2 relative logit error, top-1 identical except at near-ties); 1 (int8) is for experiments.
_ACT_LIMBS = [int(os.environ.get("SMPQ_ACT_LIMBS", "3"))]
# optional launch observer (bench.py): object with begin() / end(work) around each conv
_CONV_HOOK = [None]
LIMB_QMAX = {1: 127.0, 2: 32512.0, 3: 8323072.0}


def set_act_limbs(limbs):
    if limbs not in (1, 2, 3):
        raise ValueError("act limbs must be 1, 2 or 3")
    _ACT_LIMBS[0] = int(limbs)


def get_act_limbs():
    return _ACT_LIMBS[0]


def _req(cond, msg):
    if not cond:
        raise ValueError("smpq: " + msg)


# Rounding semantics of functions.py:41 `t / scale` (include/smpq.h SMPQ_QSEM_*): torch on the CPU
# divides (IEEE fp32), torch on the GPU multiplies by fp32(1.0 / scale). "auto" follows the
# tensor's device, as the reference's own result does; SMPQ_QUANT_SEMANTICS overrides it.
QSEM = {"cpu": 0, "device": 1}
_QSEM_MODE = [os.environ.get("SMPQ_QUANT_SEMANTICS", "auto")]


def set_quant_semantics(mode):
    """'auto' (default: device tensors round like torch on the GPU, host tensors like torch on
    the CPU), 'cpu' or 'device' (every tensor rounds that way)."""
    if mode not in ("auto", "cpu", "device"):
        raise ValueError("quant semantics must be 'auto', 'cpu' or 'device'")
    _QSEM_MODE[0] = mode


def get_quant_semantics():
    return _QSEM_MODE[0]


def _qsem(semantics, is_cuda):
    mode = semantics or _QSEM_MODE[0]
    if mode == "auto":
        mode = "device" if is_cuda else "cpu"
    _req(mode in QSEM, "quant semantics must be 'auto', 'cpu' or 'device'")
    return QSEM[mode]


def quantize_channels_(w2d, bits, semantics=None):
    """In-place fake-quantization of the rows of ``w2d`` (functions.py:25-43 per channel).

    w2d: fp32 [cout, k] contiguous (CPU or GPU); bits: int sequence/tensor [cout], 0 = skip.
    semantics: None (the process setting, ``set_quant_semantics``), 'auto', 'cpu' or 'device'.
    Returns the fp32 step (fp32(scale)) per row (0 for skipped rows) on w2d's device.
    Raises ZeroDivisionError on a constant channel, like the reference (functions.py:40).
    """
    _req(w2d.dtype == torch.float32 and w2d.dim() == 2 and w2d.is_contiguous(),
         "quantize_channels_: need a contiguous fp32 [cout, k] tensor")
    cout, k = w2d.shape
    lib = _lib.load()
    sem = _qsem(semantics, w2d.is_cuda)
    bits_t = torch.as_tensor(bits, dtype=torch.int8).reshape(-1)
    _req(bits_t.numel() == cout, "quantize_channels_: bits length != cout")
    _req(bool((bits_t >= 0).all()) and bool((bits_t <= 16).all()), "bits outside [0, 16]")
    if w2d.is_cuda:
        bits_d = bits_t.to(w2d.device)
        step = torch.zeros(cout, dtype=torch.float32, device=w2d.device)
        status = torch.zeros(1, dtype=torch.int32, device=w2d.device)
        with torch.cuda.device(w2d.device):
            _lib.check(lib.smpq_quantize_channels_ex(_lib.ptr(w2d), cout, k, _lib.ptr(bits_d),
                                                     _lib.ptr(step), _lib.ptr(status), sem,
                                                     _lib.stream_ptr()), "smpq_quantize_channels_ex")
        bad = int(status.item())  # one sync: the reference raises synchronously
        if bad:
            raise ZeroDivisionError("float division by zero (constant channel %d)" % (bad - 1))
        return step
    step = torch.zeros(cout, dtype=torch.float32)
    bits_c = bits_t.contiguous()
    rc = lib.smpq_quantize_channels_host_ex(_lib.ptr(w2d), cout, k, _lib.ptr(bits_c), _lib.ptr(step), sem)
    if rc == _lib.SMPQ_E_CONSTANT:
        raise ZeroDivisionError(_lib.last_error())
    _lib.check(rc, "smpq_quantize_channels_host_ex")
    return step


def pack_weights(w, step):
    """fp32 fake-quantized weight [cout, cin, kh, kw] -> (codes int8 [cout, kh*kw*cin], offset int32)."""
    _req(w.is_cuda and w.dtype == torch.float32 and w.dim() == 4, "pack_weights: need a CUDA fp32 4-D weight")
    w = w.contiguous()
    cout, cin, kh, kw = w.shape
    step = step.to(device=w.device, dtype=torch.float32).contiguous()
    _req(step.numel() == cout, "pack_weights: step length")
    codes = torch.empty(cout, kh * kw * cin, dtype=torch.int8, device=w.device)
    offset = torch.empty(cout, dtype=torch.int32, device=w.device)
    status = torch.zeros(2, dtype=torch.int32, device=w.device)
    lib = _lib.load()
    with torch.cuda.device(w.device):
        _lib.check(lib.smpq_pack_weights(_lib.ptr(w), cout, cin, kh, kw, _lib.ptr(step), _lib.ptr(codes),
                                         _lib.ptr(offset), _lib.ptr(status), _lib.stream_ptr()),
                   "smpq_pack_weights")
    return codes, offset, status


def pack_weights_ex(w, step, wlimbs):
    """Weight codes for conv2d_q: (codes int8 [wlimbs, cout, K], offset int32 [cout] | None,
    wscale fp32 [cout], status int32 [3] (device)). See include/smpq.h smpq_pack_weights_ex."""
    _req(w.is_cuda and w.dtype == torch.float32 and w.dim() == 4, "pack_weights_ex: need a CUDA fp32 4-D weight")
    _req(wlimbs in (1, 2, 3), "pack_weights_ex: wlimbs")
    w = w.contiguous()
    cout, cin, kh, kw = w.shape
    _req(cin % 64 == 0, "pack_weights_ex: cin must be a multiple of 64 (the stem: pack_weights_s2d)")
    K = cin * kh * kw
    if step is not None:
        step = step.to(device=w.device, dtype=torch.float32).contiguous()
        _req(step.numel() == cout, "pack_weights_ex: step length")
    _req(wlimbs >= 2 or step is not None, "pack_weights_ex: wlimbs=1 needs step")
    codes = torch.empty(wlimbs, cout, K, dtype=torch.int8, device=w.device)
    offset = torch.zeros(cout, dtype=torch.int32, device=w.device)
    wscale = torch.empty(cout, dtype=torch.float32, device=w.device)
    status = torch.zeros(3, dtype=torch.int32, device=w.device)
    lib = _lib.load()
    with torch.cuda.device(w.device):
        _lib.check(lib.smpq_pack_weights_ex(_lib.ptr(w), cout, cin, kh, kw, _lib.ptr(step), int(wlimbs),
                                            _lib.ptr(codes), _lib.ptr(offset), _lib.ptr(wscale), _lib.ptr(status),
                                            _lib.stream_ptr()), "smpq_pack_weights_ex")
    if KMAJOR[0]:
        # the K-major copy the LDS-DMA tiles stage their weight pieces from (whole cache lines);
        # it lives and dies with these codes
        codes._smpq_km = weights_kmajor(codes)
    return codes, offset, wscale, status


KMAJOR = [os.environ.get("SMPQ_KMAJOR", "1") != "0"]


def weights_kmajor(codes):
    """codes int8 [LW, cout, K] (K % 64 == 0) -> the K-major copy [LW, K/64, cout, 64]
    (smpq_weights_kmajor) that smpq_conv2d_fwd_q_km's LDS-DMA tiles read."""
    if codes.dim() == 2:
        codes = codes.unsqueeze(0)
    wl, cout, K = codes.shape
    _req(codes.is_cuda and codes.dtype == torch.int8 and codes.is_contiguous() and K % 64 == 0,
         "weights_kmajor: need contiguous int8 [LW, cout, K] with K % 64 == 0")
    out = torch.empty(wl, K // 64, cout, 64, dtype=torch.int8, device=codes.device)
    lib = _lib.load()
    with torch.cuda.device(codes.device):
        _lib.check(lib.smpq_weights_kmajor(_lib.ptr(codes), int(wl), int(cout), int(K), _lib.ptr(out),
                                           _lib.stream_ptr()), "smpq_weights_kmajor")
    return out


def image_quantize_s2d(x, x_absmax, limbs=None):
    """NCHW fp32 images (c <= 4, h, w >= 2) -> space-to-depth limb planes
    [limbs, n, ceil(h/2), ceil(w/2), 16] (channel (dy*2 + dx)*4 + c = pixel (2i+dy, 2j+dx), channel c;
    zero past an odd h or w): the stem's input (stem_conv_s2d)."""
    limbs = limbs or get_act_limbs()
    _req(x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.is_contiguous() and x.shape[1] <= 4,
         "image_quantize_s2d: need contiguous NCHW fp32 with <= 4 channels")
    n, c, h, w = x.shape
    _req(h >= 2 and w >= 2, "image_quantize_s2d: h and w must be >= 2")
    _req(x_absmax.numel() == n and x_absmax.dtype == torch.float32, "image_quantize_s2d: absmax")
    out = torch.empty(limbs, n, (h + 1) // 2, (w + 1) // 2, 16, dtype=torch.int8, device=x.device)
    lib = _lib.load()
    with torch.cuda.device(x.device):
        _lib.check(lib.smpq_image_quantize_s2d(_lib.ptr(x), n, c, h, w, _lib.ptr(x_absmax), int(limbs),
                                               _lib.ptr(out), _lib.stream_ptr()), "smpq_image_quantize_s2d")
    return out


def pack_weights_s2d(w, wlimbs, step=None):
    """7x7 stem weight fp32 [cout, c <= 4, 7, 7] -> (codes int8 [wlimbs, cout, 256] in the
    space-to-depth K order, wscale fp32 [cout]): channels with a recorded quantization step
    (``step`` [cout], 0 = never quantized) as exact codes, the others in per-channel fixed point
    (wlimbs 2 or 3: 16 / 24 bits), like pack_weights_ex."""
    _req(w.is_cuda and w.dtype == torch.float32 and w.dim() == 4 and tuple(w.shape[2:]) == (7, 7)
         and w.shape[1] <= 4, "pack_weights_s2d: need a CUDA fp32 [cout, <=4, 7, 7] weight")
    _req(wlimbs in (2, 3), "pack_weights_s2d: wlimbs must be 2 or 3")
    w = w.contiguous()
    cout, cin = w.shape[:2]
    codes = torch.empty(wlimbs, cout, 256, dtype=torch.int8, device=w.device)
    wscale = torch.empty(cout, dtype=torch.float32, device=w.device)
    status = torch.zeros(3, dtype=torch.int32, device=w.device)
    if step is not None:
        step = step.to(device=w.device, dtype=torch.float32).contiguous()
        _req(step.numel() == cout, "pack_weights_s2d: step length")
    lib = _lib.load()
    with torch.cuda.device(w.device):
        _lib.check(lib.smpq_pack_weights_s2d_ex(_lib.ptr(w), cout, cin, _lib.ptr(step), int(wlimbs), _lib.ptr(codes),
                                                _lib.ptr(wscale), _lib.ptr(status), _lib.stream_ptr()),
                   "smpq_pack_weights_s2d_ex")
    return codes, wscale


def stem_conv_s2d(xq, x_absmax, codes, h, w, col_scale, col_shift, relu=True, y_absmax=None, tile_cfg=-1,
                  emit_range=None, overflow=None, want_f32=True):
    """The stem conv (7x7/2/3 on the original h x w image) on space-to-depth planes from
    image_quantize_s2d with pack_weights_s2d codes -> NHWC fp32 y [n, h/2, w/2, cout] (and the
    next limb planes when emit_range is given: returns (y or None, yq) then)."""
    limbs, n, h2, w2, c16 = xq.shape
    _req(c16 == 16 and h2 == (h + 1) // 2 and w2 == (w + 1) // 2, "stem_conv_s2d: planes do not match h, w")
    wlimbs, cout, K = codes.shape
    _req(K == 256, "stem_conv_s2d: codes must come from pack_weights_s2d")
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    if emit_range is None:
        want_f32 = True
    y = torch.empty(n, ho, wo, cout, dtype=torch.float32, device=xq.device) if want_f32 else None
    yq = None
    if emit_range is not None:
        _req(overflow is not None, "stem_conv_s2d: emit_range needs an overflow flag tensor")
        yq = torch.empty(limbs, n, ho, wo, cout, dtype=torch.int8, device=xq.device)
    per_img = max(limbs * h2 * w2 * 16, (4 if want_f32 else 0) * ho * wo * cout,
                  (limbs if yq is not None else 0) * ho * wo * cout)
    nchunk = PLANE_LIMIT // per_img
    _req(nchunk >= 1, "stem_conv_s2d: one image's planes exceed 2 GiB")
    if n > nchunk:
        # 32-bit plane offsets in the kernel: the images in chunks, as conv2d_q does (every image
        # is independent, so the result is that of one launch)
        for i0 in range(0, n, nchunk):
            i1 = min(n, i0 + nchunk)
            r = stem_conv_s2d(xq[:, i0:i1].contiguous(), x_absmax[i0:i1], codes, h, w, col_scale, col_shift, relu,
                              None if y_absmax is None else y_absmax[i0:i1], tile_cfg, emit_range, overflow, want_f32)
            if emit_range is None:
                y[i0:i1].copy_(r)
            else:
                if y is not None:
                    y[i0:i1].copy_(r[0])
                yq[:, i0:i1].copy_(r[1])
        return y if emit_range is None else (y, yq)
    lib = _lib.load()
    hook = _CONV_HOOK[0]
    if hook is not None:
        hook.begin()
    with torch.cuda.device(xq.device):
        _lib.check(lib.smpq_stem_conv_s2d_q(
            _lib.ptr(xq), _lib.ptr(x_absmax), n, h, w, _lib.ptr(codes), int(wlimbs), cout, _lib.ptr(col_scale),
            _lib.ptr(col_shift), 1 if relu else 0, int(limbs), _lib.ptr(y), _lib.ptr(y_absmax), _lib.ptr(yq),
            float(emit_range or 0.0), _lib.ptr(overflow), int(tile_cfg), _lib.stream_ptr()), "smpq_stem_conv_s2d_q")
    if hook is not None:
        hook.end(alg_work(n, h, w, 3, cout, 7, 7, ho, wo, limbs, wlimbs, y is not None, yq is not None, False, False))
    return y if emit_range is None else (y, yq)


def tuned_stem_conv_s2d(xq, x_absmax, codes, h, w, col_scale, col_shift, relu=True, y_absmax=None, **kw):
    """stem_conv_s2d on the tile the committed table (or the autotuner) picks for this shape
    (every tile gives bitwise-identical results)."""
    key = ("stem_s2d", tuple(xq.shape), tuple(codes.shape), h, w, y_absmax is not None,
           kw.get("emit_range") is not None, kw.get("want_f32", True))

    def run(c):
        stem_conv_s2d(xq, x_absmax, codes, h, w, col_scale, col_shift, relu, y_absmax, c, **kw)
    # (the stem's 16-channel pixels use 64-wide K steps)
    cfg = _choose_tile(key, run, [c for c in tile_configs() if tile_kind(c) == TILE_LDS_DMA])
    return stem_conv_s2d(xq, x_absmax, codes, h, w, col_scale, col_shift, relu, y_absmax,
                         -1 if cfg is None else cfg, **kw)


def stem_pool_supported(xq, codes, h, w):
    """True when stem_pool_s2d handles these planes / codes (cout 64, h and w multiples of 4,
    w <= 224, (limbs, wlimbs) in {(3, 3), (2, 2), (1, 2)})."""
    limbs, n = xq.shape[:2]
    wlimbs, cout = codes.shape[:2]
    return bool(_lib.load().smpq_stem_pool_supported(n, h, w, cout, int(limbs), int(wlimbs)))


def stem_pool_s2d(xq, x_absmax, codes, h, w, col_scale, col_shift, emit_range, overflow):
    """conv1 7x7/2/3 + BN + ReLU + maxpool 3x3/2/1 (resnet.py:143-147) in one launch, static range:
    the pooled output's limb planes [limbs, n, h/4, w/4, 64], bitwise identical to
    maxpool_limbs(stem_conv_s2d(..., relu=True, emit_range=emit_range)[1])."""
    limbs, n, h2, w2, c16 = xq.shape
    _req(c16 == 16 and h2 == (h + 1) // 2 and w2 == (w + 1) // 2, "stem_pool_s2d: planes do not match h, w")
    wlimbs, cout, K = codes.shape
    _req(K == 256, "stem_pool_s2d: codes must come from pack_weights_s2d")
    _req(overflow is not None and emit_range is not None, "stem_pool_s2d: needs an output range and an overflow flag")
    yq = torch.empty(limbs, n, h // 4, w // 4, cout, dtype=torch.int8, device=xq.device)
    lib = _lib.load()
    hook = _CONV_HOOK[0]
    if hook is not None:
        hook.begin()
    with torch.cuda.device(xq.device):
        _lib.check(lib.smpq_stem_pool_s2d_q(
            _lib.ptr(xq), _lib.ptr(x_absmax), n, h, w, _lib.ptr(codes), int(wlimbs), cout, _lib.ptr(col_scale),
            _lib.ptr(col_shift), int(limbs), _lib.ptr(yq), float(emit_range), _lib.ptr(overflow),
            _lib.stream_ptr()), "smpq_stem_pool_s2d_q")
    if hook is not None:
        work = alg_work(n, h, w, 3, cout, 7, 7, h // 2, w // 2, limbs, wlimbs, False, False, False, False)
        work["bytes"] += limbs * n * (h // 4) * (w // 4) * cout  # the pooled output, written once
        work["shape"] = "%4d->%4d k7 %3d->%3d pool" % (3, cout, h, h // 4)
        hook.end(work)
    return yq


def maxpool_limbs(xq):
    """3x3/2/1 max pool on limb planes [L, n, h, w, c] (c % 16 == 0) -> [L, n, ho, wo, c] (exact:
    the quantizer is monotone, so pooling the codes = quantizing the pooled values)."""
    limbs, n, h, w, c = xq.shape
    _req(xq.is_cuda and xq.dtype == torch.int8 and xq.is_contiguous() and c % 16 == 0, "maxpool_limbs: planes")
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    out = torch.empty(limbs, n, ho, wo, c, dtype=torch.int8, device=xq.device)
    lib = _lib.load()
    with torch.cuda.device(xq.device):
        _lib.check(lib.smpq_maxpool_limbs(_lib.ptr(xq), n, h, w, c, int(limbs), _lib.ptr(out), _lib.stream_ptr()),
                   "smpq_maxpool_limbs")
    return out


def maxpool_quantize(x_nhwc, x_absmax, limbs=None, want_f32=True):
    """MaxPool2d(3, 2, 1) on NHWC fp32 fused with the activation quantizer of its output.
    Returns (limb planes [limbs, n, ho, wo, c], fp32 NHWC pooled or None)."""
    limbs = limbs or get_act_limbs()
    _req(x_nhwc.is_cuda and x_nhwc.dtype == torch.float32 and x_nhwc.dim() == 4 and x_nhwc.is_contiguous()
         and x_nhwc.shape[3] % 4 == 0, "maxpool_quantize: need contiguous NHWC fp32, c % 4 == 0")
    n, h, w, c = x_nhwc.shape
    _req(x_absmax.numel() == n and x_absmax.dtype == torch.float32, "maxpool_quantize: absmax")
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    q = torch.empty(limbs, n, ho, wo, c, dtype=torch.int8, device=x_nhwc.device)
    f = torch.empty(n, ho, wo, c, dtype=torch.float32, device=x_nhwc.device) if want_f32 else None
    lib = _lib.load()
    with torch.cuda.device(x_nhwc.device):
        _lib.check(lib.smpq_maxpool_quantize(_lib.ptr(x_nhwc), n, h, w, c, _lib.ptr(x_absmax), int(limbs), _lib.ptr(q),
                                             _lib.ptr(f), _lib.stream_ptr()), "smpq_maxpool_quantize")
    return q, f


def act_absmax(x_nhwc, out=None):
    """Per-image max|x| of an NHWC (or any [n, ...]) fp32 CUDA tensor -> fp32 [n]."""
    _req(x_nhwc.is_cuda and x_nhwc.dtype == torch.float32 and x_nhwc.is_contiguous(),
         "act_absmax: need a contiguous CUDA fp32 tensor")
    n = x_nhwc.shape[0]
    if out is None:
        out = torch.zeros(n, dtype=torch.float32, device=x_nhwc.device)
    _req(out.numel() == n and out.dtype == torch.float32 and out.is_contiguous(), "act_absmax: out")
    per = x_nhwc.numel() // n
    lib = _lib.load()
    with torch.cuda.device(x_nhwc.device):
        _lib.check(lib.smpq_act_absmax(_lib.ptr(x_nhwc), n, per, _lib.ptr(out), _lib.stream_ptr()),
                   "smpq_act_absmax")
    return out


def act_quantize(x, x_absmax, limbs=None, out=None):
    """fp32 [n, ...] -> int8 [limbs, n, ...] balanced digit planes (per-image range x_absmax)."""
    limbs = limbs or get_act_limbs()
    _req(x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(), "act_quantize: need contiguous CUDA fp32")
    n = x.shape[0]
    per = x.numel() // n
    _req(per % 8 == 0, "act_quantize: elements per image must be a multiple of 8")
    _req(x_absmax.dtype == torch.float32 and x_absmax.numel() == n and x_absmax.device == x.device, "act_quantize: absmax")
    if out is None:
        out = torch.empty((limbs,) + tuple(x.shape), dtype=torch.int8, device=x.device)
    _req(out.shape == (limbs,) + tuple(x.shape) and out.dtype == torch.int8 and out.is_contiguous(), "act_quantize: out")
    lib = _lib.load()
    with torch.cuda.device(x.device):
        _lib.check(lib.smpq_act_quantize(_lib.ptr(x), n, per, _lib.ptr(x_absmax), int(limbs), _lib.ptr(out),
                                         _lib.stream_ptr()), "smpq_act_quantize")
    return out


_TILES = {}


def tile_configs():
    """{cfg: (BM, BN, threads)} of the conv kernel's block tiles (BM output pixels x BN output
    channels; csrc/conv_glds_kernel.h kGlds)."""
    if not _TILES:
        lib = _lib.load()
        import ctypes
        for c in range(lib.smpq_conv2d_num_tile_configs()):
            bm, bn, nt = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            _lib.check(lib.smpq_conv2d_tile_config(c, ctypes.byref(bm), ctypes.byref(bn), ctypes.byref(nt)),
                       "smpq_conv2d_tile_config")
            _TILES[c] = (bm.value, bn.value, nt.value)
            kind = lib.smpq_conv2d_tile_kind(c)
            if kind < 0:
                _lib.check(kind, "smpq_conv2d_tile_kind")
            _KINDS[c] = kind
    return _TILES


TILE_LDS_DMA, TILE_LDS_DMA_K128, TILE_HALO3X3, TILE_RESIDENT1X1 = 2, 3, 4, 5  # include/smpq.h SMPQ_TILE_*
_KINDS = {}


def tile_kind(cfg):
    """Kernel family of a tile config (TILE_LDS_DMA / TILE_LDS_DMA_K128: 64- or 128-wide K steps;
    TILE_HALO3X3: the halo-patch 3x3 kernel, static-range limb-plane output only)."""
    tile_configs()
    return _KINDS[cfg]


def conv2d_q(xq, x_absmax, codes, offset, kh, kw, stride, pad, col_scale, col_shift,
             residual=None, relu=False, y_absmax=None, out=None, tile_cfg=-1,
             emit_range=None, overflow=None, want_f32=True, residual_q=None, residual_range=None,
             weight_layout="auto"):
    """Quantized conv on int8 limb planes xq [L, n, h, w, cin] (from act_quantize / maxpool_quantize /
    stem_pool_s2d / a previous conv2d_q) and weight limb planes codes [LW, cout, K] (or
    [cout, K] for LW = 1): y = conv(x, w) * s_x * col_scale + col_shift (+res) (relu), NHWC fp32.
    With ``emit_range`` (static range of the output, float) the epilogue also writes the output's
    int8 limb planes [L, n, ho, wo, cout] and sets ``overflow`` (int32 [1]) if a value exceeded the
    range; returns (y or None, yq) then. ``residual_q`` (+ ``residual_range``): the residual as
    int8 limb planes [L, n, ho, wo, cout] instead of fp32 ``residual``. ``weight_layout``: "auto"
    lets the kernel read the K-major copy pack_weights_ex attached to ``codes`` (bitwise the same
    results; only while KMAJOR is on), "rowmajor" keeps it on ``codes`` itself. A batch whose
    planes would reach 2 GiB (the kernel's 32-bit buffer offsets) runs in image chunks."""
    _req(xq.is_cuda and xq.dtype == torch.int8 and xq.dim() == 5 and xq.is_contiguous(), "conv: xq must be [L,n,h,w,c] int8")
    limbs, n, h, w, cin = xq.shape
    _req(limbs in (1, 2, 3), "conv: limbs")
    km = getattr(codes, "_smpq_km", None) if (weight_layout == "auto" and KMAJOR[0]) else None
    if codes.dim() == 2:
        codes = codes.unsqueeze(0)
    wlimbs, cout, K = codes.shape
    _req(wlimbs in (1, 2, 3) and (wlimbs < 3 or limbs == 3), "conv: weight limbs")
    _req(codes.dtype == torch.int8 and K == kh * kw * cin and codes.is_contiguous() and codes.device == xq.device,
         "conv: codes shape")
    _req(cin % 64 == 0, "conv: cin must be a multiple of 64 (the <= 4-channel stem: stem_conv_s2d)")
    _req(cout % 16 == 0, "conv: cout must be a multiple of 16")
    _req(offset is None or (offset.dtype == torch.int32 and offset.numel() == cout), "conv: offset")
    _req(x_absmax.dtype == torch.float32 and x_absmax.numel() == n, "conv: x_absmax")
    for t in (col_scale, col_shift):
        _req(t.dtype == torch.float32 and t.numel() == cout and t.is_contiguous() and t.device == xq.device,
             "conv: col vectors")
    ho = (h + 2 * pad - kh) // stride + 1
    wo = (w + 2 * pad - kw) // stride + 1
    _req(ho > 0 and wo > 0, "conv: empty output")
    yq = None
    if emit_range is not None:
        _req(emit_range > 0 and cout % 4 == 0, "conv: emit_range must be > 0 and cout % 4 == 0")
        _req(overflow is not None and overflow.dtype == torch.int32 and overflow.device == xq.device, "conv: overflow")
        yq = torch.empty(limbs, n, ho, wo, cout, dtype=torch.int8, device=xq.device)
    else:
        want_f32 = True
    if out is None and want_f32:
        out = torch.empty(n, ho, wo, cout, dtype=torch.float32, device=xq.device)
    _req(out is None or (out.shape == (n, ho, wo, cout) and out.is_contiguous()), "conv: out shape")
    if residual is not None:
        _req(residual.shape == (n, ho, wo, cout) and residual.is_contiguous() and residual.dtype == torch.float32,
             "conv: residual shape")
    if residual_q is not None:
        _req(residual is None and residual_q.shape == (limbs, n, ho, wo, cout) and residual_q.dtype == torch.int8
             and residual_q.is_contiguous() and residual_range is not None and residual_range > 0
             and cout % 4 == 0, "conv: residual_q")
    if y_absmax is not None:
        _req(y_absmax.numel() == n and y_absmax.dtype == torch.float32, "conv: y_absmax")
    per_img = max(limbs * h * w * cin, (limbs if (yq is not None or residual_q is not None) else 0) * ho * wo * cout,
                  (4 if (out is not None or residual is not None) else 0) * ho * wo * cout)
    nchunk = PLANE_LIMIT // per_img
    _req(nchunk >= 1, "conv: one image's planes exceed 2 GiB")
    if n > nchunk:
        # the kernel addresses each plane with 32-bit offsets: run the images in chunks (every
        # image is independent, so the result is the same as one launch)
        for i0 in range(0, n, nchunk):
            i1 = min(n, i0 + nchunk)
            r = conv2d_q(xq[:, i0:i1].contiguous(), x_absmax[i0:i1], codes, offset, kh, kw, stride, pad,
                         col_scale, col_shift, residual=None if residual is None else residual[i0:i1], relu=relu,
                         y_absmax=None if y_absmax is None else y_absmax[i0:i1],
                         out=None if out is None else out[i0:i1], tile_cfg=tile_cfg, emit_range=emit_range,
                         overflow=overflow, want_f32=want_f32,
                         residual_q=None if residual_q is None else residual_q[:, i0:i1].contiguous(),
                         residual_range=residual_range, weight_layout=weight_layout)
            if yq is not None:
                yq[:, i0:i1].copy_(r[1])
        return (out, yq) if emit_range is not None else out
    lib = _lib.load()
    hook = _CONV_HOOK[0]
    if hook is not None:
        hook.begin()
    with torch.cuda.device(xq.device):
        if km is not None:
            _req(km.shape == (wlimbs, K // 64, cout, 64) and km.device == xq.device, "conv: K-major codes")
        _lib.check(lib.smpq_conv2d_fwd_q_km(
            _lib.ptr(xq), _lib.ptr(x_absmax), n, h, w, cin, _lib.ptr(codes), _lib.ptr(km), int(wlimbs),
            _lib.ptr(offset), cout,
            kh, kw, stride, pad, _lib.ptr(col_scale), _lib.ptr(col_shift), _lib.ptr(residual), 1 if relu else 0,
            int(limbs), _lib.ptr(out), _lib.ptr(y_absmax), _lib.ptr(yq), float(emit_range or 0.0),
            _lib.ptr(overflow), _lib.ptr(residual_q), float(residual_range or 0.0), int(tile_cfg),
            _lib.stream_ptr()), "smpq_conv2d_fwd_q_km")
    if hook is not None:
        hook.end(alg_work(n, h, w, cin, cout, kh, kw, ho, wo, limbs, wlimbs, out is not None, yq is not None,
                          residual is not None, residual_q is not None))
    if emit_range is not None:
        return out, yq
    return out


# bytes per plane the kernel's 32-bit buffer offsets address (csrc/conv_glds.hip glds_planes_ok)
PLANE_LIMIT = 0x7fffff00


def conv_pair_supported(cin, cout1, cout2, limbs=3):
    """Does smpq_conv2d_pair_fwd run this Bottleneck chain (conv3 cin -> cout1, next conv1 cout1 ->
    cout2)?"""
    return bool(_lib.load().smpq_conv2d_pair_supported(int(cin), int(cout1), int(cout2), int(limbs)))


def conv_chain_supported(cin, cout1, cout2=0, limbs=3):
    """Does smpq_conv2d_chain_fwd run a conv3 cin -> cout1 (+ a fused downsample) (-> next conv1
    cout1 -> cout2; 0: none)?"""
    return bool(_lib.load().smpq_conv2d_chain_supported(int(cin), int(cout1), int(cout2), int(limbs)))


def conv_chain_ds_supported(cin, cout1, ds_cin, ds_stride, limbs=3):
    """Does smpq_conv2d_chain_fwd run conv3 cin -> cout1 with a fused 1x1 downsample ds_cin ->
    cout1 of this stride (and no chained conv1)?"""
    return bool(_lib.load().smpq_conv2d_chain_ds_supported(int(cin), int(cout1), int(ds_cin), int(ds_stride),
                                                           int(limbs)))


def _one_limb(codes, what):
    _req(codes.dim() == 2 or codes.shape[0] == 1, "chain: %s needs exact codes (one weight limb)" % what)
    return codes[0] if codes.dim() == 3 else codes


def conv_chain_q(xq, x_absmax, codes1, offset1, col_scale1, col_shift1, emit_range1, y1_absmax, overflow,
                 residual_q=None, residual_range=None, ds=None, nxt=None):
    """A Bottleneck's conv3 (1x1 + folded BN + identity + ReLU, exact codes, optional weight offsets)
    in one launch with (csrc/conv_resident.hip, smpq_conv2d_chain_fwd):
      - its identity: ``residual_q`` limb planes (+ ``residual_range``), or ``ds`` = (ds_xq,
        ds_x_absmax, ds_codes [3, cout1, ds_cin], ds_col_scale, ds_col_shift, ds_range[, ds_stride]):
        the block's 1x1 downsample (stride 1 by default) over conv3's output pixels, computed in the
        same tiles (its output codes feed the residual; never written);
      - ``nxt`` = (codes2, col_scale2, col_shift2, emit_range2): the next block's conv1 (ReLU) on
        conv3's output tile.
    Returns (yq1, yq2 or None), bitwise what the separate launches write; ``overflow`` covers every
    output of the chain (the downsample's included)."""
    _req(xq.is_cuda and xq.dtype == torch.int8 and xq.dim() == 5 and xq.is_contiguous(), "chain: xq")
    limbs, n, h, w, cin = xq.shape
    c1 = _one_limb(codes1, "conv3")
    cout1 = c1.shape[0]
    c2 = _one_limb(nxt[0], "conv1") if nxt is not None else None
    cout2 = c2.shape[0] if c2 is not None else 0
    _req(c1.shape == (cout1, cin) and c1.is_contiguous() and c1.dtype == torch.int8, "chain: conv3 codes")
    _req(c2 is None or (c2.shape == (cout2, cout1) and c2.is_contiguous() and c2.dtype == torch.int8),
         "chain: conv1 codes")
    ds_stride = int(ds[6]) if (ds is not None and len(ds) > 6) else 1
    if ds is not None:
        _req(cout2 == 0 and conv_chain_ds_supported(cin, cout1, ds[0].shape[-1], ds_stride, limbs),
             "chain: shape not built")
    else:
        _req(conv_chain_supported(cin, cout1, cout2, limbs), "chain: shape not built")
    _req((residual_q is None) != (ds is None), "chain: one identity source (residual_q or ds)")
    _req(offset1 is None or (offset1.dtype == torch.int32 and offset1.numel() == cout1), "chain: offset")
    if residual_q is not None:
        _req(residual_q.shape == (limbs, n, h, w, cout1) and residual_q.dtype == torch.int8
             and residual_q.is_contiguous() and residual_range is not None and residual_range > 0, "chain: residual_q")
    vecs = [(col_scale1, cout1), (col_shift1, cout1)]
    if ds is not None:
        dxq, dam, dcodes, dcs, dsh, drng = ds[:6]
        _, _, dh, dw, dcin = dxq.shape
        _req(dxq.dim() == 5 and dxq.shape[:2] == (limbs, n) and (dh - 1) // ds_stride + 1 == h
             and (dw - 1) // ds_stride + 1 == w and dxq.dtype == torch.int8 and dxq.is_contiguous()
             and dam.numel() == n, "chain: downsample input (its output pixels must be conv3's)")
        _req(dcodes.shape == (3, cout1, dcin) and dcodes.dtype == torch.int8 and dcodes.is_contiguous(),
             "chain: downsample codes [3, cout, ds_cin]")
        _req(drng > 0, "chain: downsample range")
        vecs += [(dcs, cout1), (dsh, cout1)]
    if nxt is not None:
        vecs += [(nxt[1], cout2), (nxt[2], cout2)]
        _req(y1_absmax is not None and y1_absmax.numel() == n, "chain: y1_absmax")
    for t, c in vecs:
        _req(t.dtype == torch.float32 and t.numel() == c and t.is_contiguous() and t.device == xq.device,
             "chain: col vectors")
    _req(x_absmax.numel() == n and overflow is not None and overflow.dtype == torch.int32
         and overflow.device == xq.device, "chain: absmax / overflow")
    nchunk = PLANE_LIMIT // (limbs * max(h * w * max(cin, cout1), 0 if ds is None else ds[0].shape[2] * ds[0].shape[3]
                                         * ds[0].shape[4]))
    _req(nchunk >= 1, "chain: one image's planes exceed 2 GiB")
    if n > nchunk:  # 32-bit buffer offsets: image chunks (independent images, the same result)
        yq1 = torch.empty(limbs, n, h, w, cout1, dtype=torch.int8, device=xq.device)
        yq2 = torch.empty(limbs, n, h, w, cout2, dtype=torch.int8, device=xq.device) if nxt is not None else None
        for i0 in range(0, n, nchunk):
            i1 = min(n, i0 + nchunk)
            a, b = conv_chain_q(
                xq[:, i0:i1].contiguous(), x_absmax[i0:i1], codes1, offset1, col_scale1, col_shift1, emit_range1,
                None if y1_absmax is None else y1_absmax[i0:i1], overflow,
                residual_q=None if residual_q is None else residual_q[:, i0:i1].contiguous(),
                residual_range=residual_range,
                ds=None if ds is None else (ds[0][:, i0:i1].contiguous(), ds[1][i0:i1]) + tuple(ds[2:]), nxt=nxt)
            yq1[:, i0:i1].copy_(a)
            if b is not None:
                yq2[:, i0:i1].copy_(b)
        return yq1, yq2
    yq1 = torch.empty(limbs, n, h, w, cout1, dtype=torch.int8, device=xq.device)
    yq2 = torch.empty(limbs, n, h, w, cout2, dtype=torch.int8, device=xq.device) if nxt is not None else None
    lib = _lib.load()
    hook = _CONV_HOOK[0]
    if hook is not None:
        hook.begin()
    P = _lib.ptr
    with torch.cuda.device(xq.device):
        _lib.check(lib.smpq_conv2d_chain_fwd(
            P(xq), P(x_absmax), n, h, w, cin, P(c1), P(offset1), cout1, P(col_scale1), P(col_shift1),
            P(residual_q), float(residual_range or 0.0),
            P(ds[0]) if ds else None, P(ds[1]) if ds else None, ds[0].shape[2] if ds else 0,
            ds[0].shape[3] if ds else 0, ds[0].shape[4] if ds else 0, ds_stride if ds else 0,
            P(ds[2]) if ds else None, 3 if ds else 0,
            P(ds[3]) if ds else None, P(ds[4]) if ds else None, float(ds[5]) if ds else 0.0,
            P(yq1), float(emit_range1), P(y1_absmax),
            P(c2), cout2, P(nxt[1]) if nxt else None, P(nxt[2]) if nxt else None, P(yq2),
            float(nxt[3]) if nxt else 0.0, P(overflow), _lib.stream_ptr()), "smpq_conv2d_chain_fwd")
    if hook is not None:
        # one launch doing every chained conv's work; the reads / writes it removes are not counted
        w1 = alg_work(n, h, w, cin, cout1, 1, 1, h, w, limbs, 1, False, True, False, residual_q is not None)
        ops_, nbytes, shape = w1["ops"], w1["bytes"], "%4d->%4d" % (cin, cout1)
        if ds is not None:
            wd = alg_work(n, ds[0].shape[2], ds[0].shape[3], ds[0].shape[4], cout1, 1, 1, h, w, limbs, 3, False,
                          False, False, False)
            ops_ += wd["ops"]
            nbytes += wd["bytes"]  # the downsample's input and weights (its output never leaves the CU)
            shape += "+ds"
        if nxt is not None:
            w2 = alg_work(n, h, w, cout1, cout2, 1, 1, h, w, limbs, 1, False, True, False, False)
            ops_ += w2["ops"]
            nbytes += w2["bytes"] - limbs * n * h * w * cout1  # conv1 reads conv3's tile from LDS
            shape += "->%4d" % cout2
        hook.end({"ops": ops_, "bytes": nbytes, "passes": w1["passes"], "shape": "%s k1 %3d chain" % (shape, h)})
    return yq1, yq2


def conv_pair_q(xq, x_absmax, codes1, col_scale1, col_shift1, residual_q, residual_range, emit_range1,
                y1_absmax, codes2, col_scale2, col_shift2, emit_range2, overflow):
    """A Bottleneck's conv3 (1x1 + folded BN + limb-plane identity + ReLU) chained with the next
    block's conv1 (1x1 + folded BN + ReLU) in one launch: returns (yq1, yq2), bitwise

        _, yq1 = conv2d_q(xq, x_absmax, codes1, None, 1, 1, 1, 0, col_scale1, col_shift1, relu=True,
                          emit_range=emit_range1, overflow=overflow, want_f32=False,
                          residual_q=residual_q, residual_range=residual_range)
        _, yq2 = conv2d_q(yq1, y1_absmax, codes2, None, 1, 1, 1, 0, col_scale2, col_shift2, relu=True,
                          emit_range=emit_range2, overflow=overflow, want_f32=False)

    without reading yq1 back from HBM (conv_chain_q with the next conv and no downsample)."""
    c1, c2 = _one_limb(codes1, "conv3"), _one_limb(codes2, "conv1")
    _req(conv_pair_supported(xq.shape[-1], c1.shape[0], c2.shape[0], xq.shape[0]), "pair: shape not built")
    return conv_chain_q(xq, x_absmax, codes1, None, col_scale1, col_shift1, emit_range1, y1_absmax, overflow,
                        residual_q=residual_q, residual_range=residual_range,
                        nxt=(codes2, col_scale2, col_shift2, emit_range2))


# ---- per-shape tile choice (cf. cudnn.benchmark=True, resnet50_main.py:10) ---------------------
# Every tile configuration gives bitwise-identical results; only the time differs. A shape's tile
# comes from (1) this process's cache, (2) the committed table smpq/data/tiles_gfx950.json
# (tools/tune_tiles.py: medians of many timed launches on an MI355X, so a benchmark does not depend
# on a short timing race), or (3) the autotuner: TUNE_REPS timed launches per candidate after two
# warm-ups, the candidate with the smallest median wins. SMPQ_TILE_TABLE=<path> uses another table,
# SMPQ_TILE_TABLE=off none; SMPQ_AUTOTUNE=0 turns (3) off (the C-ABI default tile then).
AUTOTUNE = [os.environ.get("SMPQ_AUTOTUNE", "1") != "0"]
TUNE_REPS = [int(os.environ.get("SMPQ_TUNE_REPS", "10"))]
# diagnostics (A/B of tile families on one box): tile configs the autotuner never tries
TILES_EXCLUDED = {int(c) for c in os.environ.get("SMPQ_TILES_EXCLUDE", "").split(",") if c.strip()}
# tools/tune_tiles.py --concurrent: time each candidate as TUNE_CONCURRENT copies launched together on
# their own streams (the timed forward runs its batch slices concurrently, and a tile's isolated time
# does not predict how it shares the GPU with the other slice's kernels); TUNE_LOG keeps every
# candidate's median per key
TUNE_CONCURRENT = [1]
TUNE_LOG = {}
_TUNED = {}
TILE_TABLE_DEFAULT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "tiles_gfx950.json")
_TABLE = {"path": None, "sha16": None, "entries": {}, "hits": 0, "tuned": 0}


def key_str(key):
    """The table's text form of a tile key (the tuple tuned_conv2d_q / tuned_stem_conv_s2d use)."""
    def f(v):
        if isinstance(v, tuple):
            return "x".join(f(u) for u in v)
        return str(int(v)) if isinstance(v, bool) else str(v)
    return "|".join(f(v) for v in key)


def load_tile_table(path=None):
    """(Re)load the committed tile table (None: SMPQ_TILE_TABLE or the default; "off": none)."""
    import hashlib
    import json
    path = path or os.environ.get("SMPQ_TILE_TABLE", TILE_TABLE_DEFAULT)
    _TABLE.update(path=None, sha16=None, entries={}, hits=0, tuned=0, loaded=True)
    if path in ("off", "0", "") or not os.path.exists(path):
        return _TABLE
    raw = open(path, "rb").read()
    doc = json.loads(raw)
    _TABLE.update(path=path, sha16=hashlib.sha256(raw).hexdigest()[:16],
                  entries={k: int(v) for k, v in doc.get("tiles", {}).items()})
    return _TABLE


def tile_table_info():
    """What the bench reports: table file, content hash, entries, table hits / autotuned shapes."""
    return {"path": None if _TABLE["path"] is None else os.path.relpath(_TABLE["path"], os.path.dirname(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))))),
            "sha16": _TABLE["sha16"], "entries": len(_TABLE["entries"]), "hits": _TABLE["hits"],
            "autotuned": _TABLE["tuned"]}


def _choose_tile(key, run, cands, variant=None):
    """The tile for ``key``: cached, from the table, or autotuned (None: the C-ABI default).
    ``variant`` separates calls of one key whose candidate sets differ (the cache only)."""
    ckey = key if variant is None else (key, variant)
    cfg = _TUNED.get(ckey)
    if cfg is not None:
        return cfg
    if not _TABLE.get("loaded"):
        load_tile_table()
    t = _TABLE["entries"].get(key_str(key))
    if t is not None and t in cands:
        _TUNED[ckey] = t
        _TABLE["hits"] += 1
        return t
    if not AUTOTUNE[0] or torch.cuda.is_current_stream_capturing():
        return None
    best = None
    nconc = TUNE_CONCURRENT[0]
    side = [torch.cuda.Stream() for _ in range(nconc)] if nconc > 1 else []

    def once(c):
        if not side:
            run(c)
            return
        main = torch.cuda.current_stream()
        for st in side:  # the copies write the same outputs: identical values, timing only
            st.wait_stream(main)
            with torch.cuda.stream(st):
                run(c)
        for st in side:
            main.wait_stream(st)
    log = TUNE_LOG.setdefault(key_str(key) + ("" if variant is None else "|" + str(variant)), {})
    for c in cands:
        if c in TILES_EXCLUDED:
            continue
        try:
            once(c)
            once(c)
            evs = []
            for _ in range(TUNE_REPS[0]):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                once(c)
                e1.record()
                evs.append((e0, e1))
        except _lib.SmpqError:
            continue  # the configuration does not take this shape
        torch.cuda.synchronize()
        ts = sorted(a.elapsed_time(b) for a, b in evs)
        t_med = ts[len(ts) // 2]
        log[c] = round(t_med * 1e3, 2)
        if best is None or t_med < best[0]:
            best = (t_med, c)
    if best is None:
        return None
    _TUNED[ckey] = best[1]
    _TABLE["tuned"] += 1
    return best[1]


def _tile_fits(cfg, limbs, wlimbs=1, cout=None, cin=None, k=1):
    """Can tile config ``cfg`` run this conv (libsmpq's own launch rules)? ``cin``/``cout`` default
    to a shape every configuration takes."""
    cin = cin if cin is not None else 128
    cout = cout if cout is not None else 64
    return bool(_lib.load().smpq_conv2d_tile_supported(int(cfg), int(cin), int(cout), int(k), int(k),
                                                         int(limbs), int(wlimbs)))


def tuned_conv2d_q(xq, x_absmax, codes, offset, kh, kw, stride, pad, col_scale, col_shift,
                   residual=None, relu=False, y_absmax=None, out=None, emit_range=None, overflow=None,
                   want_f32=True, residual_q=None, residual_range=None):
    """conv2d_q on the tile the committed table (or the autotuner) picks for this shape. Every
    tile gives bitwise-identical results (exact integer accumulation, same epilogue)."""
    limbs, n, h, w, cin = xq.shape
    wlimbs = codes.shape[0] if codes.dim() == 3 else 1
    cout = codes.shape[-2]
    key = (n, h, w, cin, cout, kh, kw, stride, pad, limbs, wlimbs, residual is not None, emit_range is not None,
           want_f32, residual_q is not None)

    def run(c):
        conv2d_q(xq, x_absmax, codes, offset, kh, kw, stride, pad, col_scale, col_shift,
                 residual=residual, relu=relu, y_absmax=y_absmax, out=out, tile_cfg=c,
                 emit_range=emit_range, overflow=overflow, want_f32=want_f32,
                 residual_q=residual_q, residual_range=residual_range)
    # the halo tiles run only the static-range limb-plane epilogue with ReLU, optionally with a
    # limb-plane residual (stride 1 / pad 1 for now): the key does not carry relu / y_absmax, so
    # other calls of a key never see them
    halo_ok = bool(relu and emit_range is not None and not want_f32 and residual is None
                   and y_absmax is None and out is None and kh == 3 and kw == 3 and stride == 1 and pad == 1)
    # the weight-stationary 1x1 tiles: the static-range limb-plane epilogue, built for the
    # downsamples (3 weight limbs, no ReLU or residual) and for exact-code convs with ReLU + a
    # limb-plane residual, ReLU only (both also with weight offsets), or neither
    # (smpq_conv2d_tile_supported checks the shape)
    res_ok = bool(emit_range is not None and not want_f32 and residual is None and y_absmax is None
                  and out is None and kh == 1 and kw == 1 and pad == 0
                  and (offset is None or (wlimbs == 1 and relu))
                  and (not (relu or residual_q is not None) if wlimbs == 3 else (relu or residual_q is None)))
    cands = [c for c in tile_configs() if _tile_fits(c, limbs, wlimbs, cout, cin, kh)
             and (halo_ok or tile_kind(c) != TILE_HALO3X3) and (res_ok or tile_kind(c) != TILE_RESIDENT1X1)]
    cfg = _choose_tile(key, run, cands, variant=None if (halo_ok or res_ok) else "nohalo")
    return conv2d_q(xq, x_absmax, codes, offset, kh, kw, stride, pad, col_scale, col_shift,
                    residual=residual, relu=relu, y_absmax=y_absmax, out=out,
                    tile_cfg=-1 if cfg is None else cfg, emit_range=emit_range, overflow=overflow,
                    want_f32=want_f32, residual_q=residual_q, residual_range=residual_range)


def conv2d_nhwc(x, x_absmax, codes, offset, kh, kw, stride, pad, col_scale, col_shift,
                residual=None, relu=False, limbs=None, y_absmax=None, out=None):
    """act_quantize + (autotuned) conv2d_q on an NHWC fp32 input."""
    xq = act_quantize(x, x_absmax, limbs)
    return tuned_conv2d_q(xq, x_absmax, codes, offset, kh, kw, stride, pad, col_scale, col_shift,
                          residual=residual, relu=relu, y_absmax=y_absmax, out=out)


def set_conv_hook(hook):
    """hook.begin() / hook.end(work) around every quantized-conv launch (bench.py's timer);
    work = alg_work(...) of the launch."""
    _CONV_HOOK[0] = hook


def alg_work(n, h, w, cin, cout, kh, kw, ho, wo, limbs, wlimbs, y_f32, y_q, res_f32, res_q):
    """Algorithmic work of one quantized-conv launch: ops = 2 * MACs; bytes =
    each input activation code read once (limbs bytes per element: the int8/16/24 code), the
    weight codes once, and every output element written once (limbs bytes for the next conv's
    limb planes, 4 for fp32) plus its residual read once (limbs or 4 bytes). Halo re-reads of
    3x3 windows and zero padding are not counted: they are the kernel's overhead."""
    macs = n * ho * wo * cout * kh * kw * cin
    out_elems = n * ho * wo * cout
    per_out = (4 if y_f32 else 0) + (limbs if y_q else 0) + (4 if res_f32 else 0) + (limbs if res_q else 0)
    # a strided 1x1 conv reads only the pixels it samples (1/stride^2 of its input)
    in_elems = n * ho * wo * cin if (kh == 1 and kw == 1) else n * h * w * cin
    nbytes = limbs * in_elems + wlimbs * cout * kh * kw * cin + out_elems * per_out
    return {"ops": 2 * macs, "bytes": nbytes, "passes": limbs * wlimbs - _skipped_passes(limbs, wlimbs),
            "shape": "%4d->%4d k%d %3d->%3d %s%s" % (cin, cout, kh, h, ho, "f" if y_f32 else "-",
                                                    "r" if (res_f32 or res_q) else "-")}


def _skipped_passes(limbs, wlimbs):
    smin = max(0, limbs + wlimbs - 4)  # low-digit products skipped by the kernels (conv.hip)
    return sum(1 for la in range(limbs) for lw in range(wlimbs) if la + lw < smin)


def debug_mfma_i8(a, b):
    """One v_mfma_i32_16x16x64_i8 with the kernel's fragment mapping: a[16,64] @ b[16,64]^T."""
    _req(a.is_cuda and a.dtype == torch.int8 and a.shape == (16, 64), "debug_mfma: a")
    _req(b.is_cuda and b.dtype == torch.int8 and b.shape == (16, 64), "debug_mfma: b")
    c = torch.empty(16, 16, dtype=torch.int32, device=a.device)
    lib = _lib.load()
    with torch.cuda.device(a.device):
        _lib.check(lib.smpq_debug_mfma_i8(_lib.ptr(a.contiguous()), _lib.ptr(b.contiguous()), _lib.ptr(c),
                                          _lib.stream_ptr()), "smpq_debug_mfma_i8")
    return c


# ---- evaluation reductions (functions.py:84-149) on device -----------------------------------
def softmax_xent(logits, labels, stats, want_probs=True):
    """One batch of functions.evaluate_acc_loss_softmax (functions.py:113-121) in one kernel:
    returns the softmax [B, C] fp32 (or None) and accumulates into ``stats`` (float64 [4], on the
    logits' device): [0] += batch-mean cross entropy, [1] += correct top-1, [2] += rows, [3] += 1."""
    _req(logits.is_cuda and logits.dtype == torch.float32 and logits.dim() == 2 and logits.is_contiguous(),
         "softmax_xent: logits must be a contiguous fp32 [B, C] device tensor")
    rows, cols = logits.shape
    labels = labels.to(device=logits.device, dtype=torch.int64).contiguous()
    _req(labels.numel() == rows, "softmax_xent: labels")
    _req(stats.dtype == torch.float64 and stats.numel() >= 4 and stats.device == logits.device, "softmax_xent: stats")
    probs = torch.empty_like(logits) if want_probs else None
    ws = torch.empty(2 * max(rows, 1), dtype=torch.float32, device=logits.device)
    with torch.cuda.device(logits.device):
        _lib.check(_lib.load().smpq_softmax_xent(_lib.ptr(logits), _lib.ptr(labels), rows, cols, _lib.ptr(probs),
                                                 _lib.ptr(stats), _lib.ptr(ws), _lib.stream_ptr()),
                   "smpq_softmax_xent")
    return probs


def kl_rows(p_ref, p, stats):
    """functions.KLdiv (functions.py:131-149) for one batch pair: stats (float64 [2]) +=
    (sum over images of sum_c p_ref * log(p_ref / p), images)."""
    for t in (p_ref, p):
        _req(t.is_cuda and t.dtype == torch.float32 and t.dim() == 2, "kl_rows: fp32 [B, C] device tensors")
    _req(p_ref.shape == p.shape and p_ref.device == p.device, "kl_rows: shapes")
    p_ref, p = p_ref.contiguous(), p.contiguous()
    _req(stats.dtype == torch.float64 and stats.numel() >= 2 and stats.device == p.device, "kl_rows: stats")
    rows, cols = p.shape
    ws = torch.empty(max(rows, 1), dtype=torch.float32, device=p.device)
    with torch.cuda.device(p.device):
        _lib.check(_lib.load().smpq_kl_rows(_lib.ptr(p_ref), _lib.ptr(p), rows, cols, _lib.ptr(stats), _lib.ptr(ws),
                                            _lib.stream_ptr()), "smpq_kl_rows")


def avgpool_fc(x_nhwc, weight, bias, out=None):
    """AdaptiveAvgPool2d(1) + flatten + Linear (resnet.py:216-218) on the last block's NHWC fp32
    output [n, h, w, c] -> logits [n, nout] fp32 (into ``out`` when given: a contiguous [n, nout]
    fp32 tensor, e.g. a batch slice's rows of the whole batch's logits). Each logit is summed in an
    order fixed by c alone (smpq_avgpool_fc), so an image's logits are the same bits in any batch
    or data-parallel shard."""
    _req(x_nhwc.is_cuda and x_nhwc.dtype == torch.float32 and x_nhwc.dim() == 4 and x_nhwc.is_contiguous(),
         "avgpool_fc: need contiguous NHWC fp32 on the GPU")
    n, h, w, c = x_nhwc.shape
    _req(c % 4 == 0, "avgpool_fc: channels must be a multiple of 4")
    wt = weight.detach().float().contiguous()
    _req(wt.dim() == 2 and wt.shape[1] == c and wt.device == x_nhwc.device, "avgpool_fc: weight shape")
    nout = wt.shape[0]
    b = None if bias is None else bias.detach().float().contiguous()
    _req(b is None or (b.numel() == nout and b.device == x_nhwc.device), "avgpool_fc: bias")
    pooled = torch.empty(n, c, dtype=torch.float32, device=x_nhwc.device)
    if out is None:
        out = torch.empty(n, nout, dtype=torch.float32, device=x_nhwc.device)
    _req(out.shape == (n, nout) and out.dtype == torch.float32 and out.is_contiguous() and out.device == x_nhwc.device,
         "avgpool_fc: out must be a contiguous [n, nout] fp32 tensor on the input's device")
    with torch.cuda.device(x_nhwc.device):
        _lib.check(_lib.load().smpq_avgpool_fc(_lib.ptr(x_nhwc), n, h * w, c, _lib.ptr(wt), _lib.ptr(b), nout,
                                               _lib.ptr(pooled), _lib.ptr(out), _lib.stream_ptr()),
                   "smpq_avgpool_fc")
    return out
