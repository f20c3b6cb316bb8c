"""GPU parity tests (run on the MI355X box with -m gpu). Every call goes through libsmpq's C-ABI.

Conv-level parity has two checks per case:
  * vs an exact emulation of the integer path (same activation codes, int GEMM in float64,
    which is exact for |sum| < 2^53): differences only from the fp32 epilogue, bound 2e-6
    relative to the magnitude of the terms;
  * vs the float64 oracle conv on the unquantized activations: bounded by the activation
    quantization error 0.5 * s_x * sum|w| per output (+ fp32 noise).
Model-level parity: logits of the fused HIP forward vs the reference's CPU logits (goldens
from the reference itself), top-1 identical; tolerance per activation width.
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

LIMB_QMAX = {1: 127.0, 2: 32512.0, 3: 8323072.0}
# max |logit - reference logit| / max |reference logit| accepted per activation width
LOGIT_RTOL = {1: 0.35, 2: 1.5e-2, 3: 2e-4}


# ----------------------------------------------------------------------------------------------
def test_mfma_i8_fragment_mapping(gpu):
    from smpq import ops
    g = torch.Generator().manual_seed(0)
    a = torch.randint(-128, 128, (16, 64), generator=g, dtype=torch.int8)
    b = torch.randint(-128, 128, (16, 64), generator=g, dtype=torch.int8)
    c = ops.debug_mfma_i8(a.to(gpu), b.to(gpu)).cpu().numpy()
    ref = a.numpy().astype(np.int64) @ b.numpy().astype(np.int64).T
    np.testing.assert_array_equal(c, ref)


def test_device_quantizer_bitexact_vs_reference(gpu):
    # CPU semantics on the device: the reference's CPU goldens
    from smpq import ops
    from test_oracle_golden import kat_cases
    for kind, chain, x, y in kat_cases():
        w = torch.from_numpy(x.copy()).reshape(1, -1).to(gpu)
        for b in chain:
            ops.quantize_channels_(w, [b], semantics="cpu")
        assert np.array_equal(w.cpu().numpy().ravel().view(np.uint32), y.view(np.uint32)), (kind, chain)
    with pytest.raises(ZeroDivisionError):
        ops.quantize_channels_(torch.full((1, 9), 0.25, device=gpu), [8])


def test_device_quantizer_matches_torch_on_gpu(gpu):
    # default semantics on a device tensor = what torch itself computes for functions.py:41 on the
    # GPU: the committed device KAT, and torch run live on this box over fresh random channels
    from smpq import ops
    import functions
    from test_oracle_golden import device_kat_cases
    for kind, chain, x, y in device_kat_cases():
        w = torch.from_numpy(x.copy()).reshape(1, -1).to(gpu)
        for b in chain:
            ops.quantize_channels_(w, [b])
        assert np.array_equal(w.cpu().numpy().ravel().view(np.uint32), y.view(np.uint32)), (kind, chain)
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_device_kat import quantize_wgt_torch
    g = torch.Generator().manual_seed(77)
    for i in range(200):
        t = (torch.randn((9, 64, 576, 1152)[i % 4], generator=g) * 0.05).to(gpu)
        b = (8, 6, 4, 2)[(i // 4) % 4]
        exp = quantize_wgt_torch(t, b)
        got = functions.quantize_wgt(t, b)
        assert torch.equal(got.view(torch.int32), exp.view(torch.int32)), (i, b)


def test_device_quantizer_layer_matches_host(gpu):
    from smpq import ops
    g = torch.Generator().manual_seed(5)
    w = torch.randn(300, 576, generator=g) * 0.05
    bits = torch.randint(0, 5, (300,), generator=g) * 2  # 0 (skip), 2, 4, 6, 8
    for sem in ("cpu", "device"):
        wd = w.clone().to(gpu)
        sd = ops.quantize_channels_(wd, bits, semantics=sem)
        wh = w.clone()
        sh = ops.quantize_channels_(wh, bits, semantics=sem)
        assert torch.equal(wd.cpu().view(torch.int32), wh.view(torch.int32)), sem
        assert torch.equal(sd.cpu(), sh), sem


@pytest.mark.parametrize("limbs", [1, 2, 3])
def test_act_quantize_digits(gpu, limbs):
    from smpq import ops
    g = torch.Generator().manual_seed(limbs)
    x = torch.randn(3, 5, 7, 64, generator=g) * torch.tensor([1.0, 30.0, 1e-3]).reshape(3, 1, 1, 1)
    x[2] = 0.0  # an all-zero image (absmax 0) quantizes to 0
    xd = x.to(gpu)
    am = ops.act_absmax(xd)
    q = ops.act_quantize(xd, am, limbs).cpu().numpy().astype(np.int64)
    assert q.shape == (limbs, 3, 5, 7, 64) and q.min() >= -128 and q.max() <= 127
    val = sum(q[l] * 256 ** l for l in range(limbs))
    qmax = np.float32(LIMB_QMAX[limbs])
    amn = am.cpu().numpy()
    inv = np.where(amn > 0, qmax / np.where(amn > 0, amn, 1).astype(np.float32), 0).astype(np.float32)
    exp = np.clip(np.rint((x.numpy() * inv[:, None, None, None]).astype(np.float32)), -qmax, qmax)
    np.testing.assert_array_equal(val, exp.astype(np.int64))
    assert np.abs(val[:2]).max() == int(qmax)


# ----------------------------------------------------------------------------------------------
def make_layer(gpu, cin, cout, k, seed, bits_choice=(8, 6, 4)):
    from smpq import ops
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cout * k * k)) ** 0.5)
    bits = torch.tensor(bits_choice)[torch.randint(0, len(bits_choice), (cout,), generator=g)]
    wd = w.to(gpu).contiguous()
    step = ops.quantize_channels_(wd.reshape(cout, -1), bits)
    codes, offset, status = ops.pack_weights(wd, step)
    assert status.cpu().tolist() == [0, 0]
    return wd, step, codes, offset


def im2col_nhwc(x, k, stride, pad):
    n, h, w, c = x.shape
    xp = np.pad(x, ((0, 0), (pad, pad), (pad, pad), (0, 0)))
    ho = (h + 2 * pad - k) // stride + 1
    wo = (w + 2 * pad - k) // stride + 1
    cols = np.empty((n, ho, wo, k, k, c), dtype=x.dtype)
    for r in range(k):
        for q in range(k):
            cols[:, :, :, r, q, :] = xp[:, r:r + stride * ho:stride, q:q + stride * wo:stride, :]
    return cols.reshape(n * ho * wo, k * k * c), ho, wo


def emulate(x, absmax, m_full, kh, stride, pad, col_scale, col_shift, residual, relu, limbs):
    """Exact emulation of the kernel's integer path (float64 GEMM of int values is exact here)."""
    qmax = np.float32(LIMB_QMAX[limbs])
    n = x.shape[0]
    with np.errstate(divide="ignore"):
        inv = np.where(absmax > 0, qmax / absmax.astype(np.float32), np.float32(0)).astype(np.float32)
    q = np.rint((x * inv[:, None, None, None]).astype(np.float32))
    q = np.clip(q, -qmax, qmax).astype(np.int64)
    digits = []
    for _ in range(limbs - 1):
        lo = ((q + 128) & 255) - 128
        digits.append(lo)
        q = (q - lo) >> 8
    digits.append(q)
    terms = []
    for l, d in enumerate(digits):
        cols, ho, wo = im2col_nhwc(d.astype(np.float64), kh, stride, pad)
        terms.append(cols @ m_full.T.astype(np.float64) * (256.0 ** l))
    v = sum(terms)
    mag = sum(np.abs(t) for t in terms)
    rscale = (absmax.astype(np.float32) * np.float32(1.0 / LIMB_QMAX[limbs])).astype(np.float64)
    rs = np.repeat(rscale, ho * wo)[:, None]
    y = v * rs * col_scale[None, :] + col_shift[None, :]
    bound = mag * rs * np.abs(col_scale[None, :]) + np.abs(col_shift[None, :])
    if residual is not None:
        y = y + residual.reshape(y.shape)
        bound = bound + np.abs(residual.reshape(y.shape))
    if relu:
        y = np.maximum(y, 0)
    return y.reshape(n, ho, wo, -1), bound.reshape(n, ho, wo, -1)


R18_SHAPES = [(64, 64, 3, 1, 56), (64, 128, 3, 2, 56), (128, 128, 3, 1, 28), (128, 256, 3, 2, 28),
              (256, 256, 3, 1, 14), (256, 512, 3, 2, 14), (512, 512, 3, 1, 7)]
R50_SHAPES = [(64, 64, 1, 1, 56), (64, 64, 3, 1, 56), (64, 256, 1, 1, 56), (256, 64, 1, 1, 56),
              (256, 128, 1, 1, 56), (128, 128, 3, 2, 56), (128, 512, 1, 1, 28), (512, 128, 1, 1, 28),
              (128, 128, 3, 1, 28), (512, 256, 1, 1, 28), (256, 256, 3, 2, 28), (256, 1024, 1, 1, 14),
              (1024, 256, 1, 1, 14), (256, 256, 3, 1, 14), (1024, 512, 1, 1, 14), (512, 512, 3, 2, 14),
              (512, 2048, 1, 1, 7), (2048, 512, 1, 1, 7), (512, 512, 3, 1, 7)]
EDGE_SHAPES = [(64, 80, 3, 2, 9), (128, 48, 1, 2, 15), (192, 112, 3, 1, 5), (64, 16, 3, 1, 1)]


def run_conv_case(gpu, cin, cout, k, stride, hin, limbs, seed, signed=False, residual=False, relu=False, batch=2):
    from smpq import ops
    wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed)
    pad = k // 2
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(batch, hin, hin, cin, generator=g)
    if not signed:
        x = torch.relu(x)
    x[min(1, batch - 1)] *= 7.0  # different per-image ranges
    xd = x.to(gpu)
    amax = ops.act_absmax(xd)
    np.testing.assert_array_equal(amax.cpu().numpy(), x.abs().amax(dim=(1, 2, 3)).numpy())
    col_scale = (step * torch.linspace(0.5, 1.5, cout, device=gpu)).contiguous()
    col_shift = torch.linspace(-0.1, 0.1, cout, device=gpu).contiguous()
    ho = (hin + 2 * pad - k) // stride + 1
    res = torch.randn(batch, ho, ho, cout, generator=g).to(gpu) if residual else None
    yam = torch.zeros(batch, device=gpu)
    y = ops.conv2d_nhwc(xd, amax, codes, offset, k, k, stride, pad, col_scale, col_shift,
                        residual=res, relu=relu, limbs=limbs, y_absmax=yam)
    torch.cuda.synchronize()
    yk = y.cpu().numpy().astype(np.float64)
    # integer-path emulation
    m_full = (codes.cpu().numpy().astype(np.int64) + offset.cpu().numpy().astype(np.int64)[:, None])
    ye, bound = emulate(x.numpy(), amax.cpu().numpy(), m_full, k, stride, pad, col_scale.cpu().numpy().astype(np.float64),
                        col_shift.cpu().numpy().astype(np.float64), None if res is None else res.cpu().numpy().astype(np.float64),
                        relu, limbs)
    err = np.abs(yk - ye)
    assert (err <= 2e-6 * bound + 1e-30).all(), ("emulation mismatch", float((err / (bound + 1e-30)).max()))
    # fp64 oracle on unquantized activations (conv with the fake-quantized fp32 weights)
    w_oracle = wd.cpu().numpy().astype(np.float64)  # fl32(m*step): exactly the reference weight
    wk = w_oracle.transpose(0, 2, 3, 1).reshape(cout, -1)
    cols, _, _ = im2col_nhwc(x.numpy().astype(np.float64), k, stride, pad)
    conv = cols @ wk.T
    cs = (col_scale.cpu().numpy().astype(np.float64) / step.cpu().numpy().astype(np.float64))
    yt = conv * cs[None, :] + col_shift.cpu().numpy()[None, :]
    if res is not None:
        yt = yt + res.cpu().numpy().reshape(yt.shape)
    if relu:
        yt = np.maximum(yt, 0)
    sx = np.repeat(amax.cpu().numpy() / LIMB_QMAX[limbs], ho * ho)[:, None]
    qbound = 0.5 * sx * (np.abs(cols) > -1).astype(np.float64) @ np.abs(wk).T * np.abs(cs)[None, :] * 1.0001
    qbound = qbound + 1e-5 * np.abs(yt) + 1e-6
    assert (np.abs(yk.reshape(yt.shape) - yt) <= qbound).all()
    # fused absmax output
    ya = np.abs(yk).reshape(batch, -1).max(1)
    np.testing.assert_array_equal(yam.cpu().numpy(), ya.astype(np.float32))
    return offset


@pytest.mark.parametrize("shape", R18_SHAPES + R50_SHAPES, ids=lambda s: "c%d_o%d_k%d_s%d_h%d" % s)
def test_conv_shapes_int16(gpu, shape):
    cin, cout, k, s, h = shape
    run_conv_case(gpu, cin, cout, k, s, h, limbs=2, seed=cin + cout + k)


@pytest.mark.parametrize("limbs", [1, 2, 3])
@pytest.mark.parametrize("shape", [(64, 64, 3, 1, 56), (256, 1024, 1, 1, 14), (512, 512, 3, 2, 14)] + EDGE_SHAPES,
                         ids=lambda s: "c%d_o%d_k%d_s%d_h%d" % s)
def test_conv_limbs_and_edges(gpu, shape, limbs):
    cin, cout, k, s, h = shape
    run_conv_case(gpu, cin, cout, k, s, h, limbs=limbs, seed=7 * cin + cout, signed=True, residual=True, relu=True, batch=3)


# tile kinds that run only the static-range limb-plane epilogue (fp32 outputs / fp32 residuals /
# 1-2 limbs: test_gpu_halo.py, test_gpu_resident.py cover them against the LDS-DMA kernel)
_LEAN_ONLY = (4, 5)  # ops.TILE_HALO3X3, ops.TILE_RESIDENT1X1


@pytest.mark.parametrize("limbs", [1, 2, 3])
@pytest.mark.parametrize("shape", [(64, 256, 1, 1, 20), (128, 128, 3, 2, 17), (64, 80, 3, 1, 9), (256, 48, 1, 1, 7)],
                         ids=lambda s: "c%d_o%d_k%d_s%d_h%d" % s)
def test_all_tile_configs_bitwise_identical(gpu, shape, limbs):
    from smpq import ops
    cin, cout, k, s, h = shape
    wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin + 3 * cout)
    x = torch.randn(3, h, h, cin, generator=torch.Generator().manual_seed(9)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    ho = (h + 2 * (k // 2) - k) // s + 1
    res = torch.randn(3, ho, ho, cout, generator=torch.Generator().manual_seed(10)).to(gpu)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    outs = []
    for c in ops.tile_configs():  # (the halo kernel runs the lean epilogue only: test_gpu_halo.py)
        if not ops._tile_fits(c, limbs, 1, cout, cin, k) or ops.tile_kind(c) in _LEAN_ONLY:
            continue
        ya = torch.zeros(3, device=gpu)
        y = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, residual=res, relu=True,
                         y_absmax=ya, tile_cfg=c)
        outs.append((c, y, ya))
    assert len(outs) >= 3
    assert any(ops.tile_kind(c) == ops.TILE_LDS_DMA for c, _, _ in outs)
    assert (cin % 128 != 0) or any(ops.tile_kind(c) == ops.TILE_LDS_DMA_K128 for c, _, _ in outs)
    for c, y, ya in outs[1:]:
        assert torch.equal(y, outs[0][1]), c
        assert torch.equal(ya, outs[0][2]), c


@pytest.mark.parametrize("range_frac", [2.0, 0.5])
@pytest.mark.parametrize("limbs", [1, 2, 3])
@pytest.mark.parametrize("shape", [(64, 256, 1, 1, 20), (128, 64, 3, 2, 17), (64, 80, 3, 1, 9)],
                         ids=lambda s: "c%d_o%d_k%d_s%d_h%d" % s)
def test_static_outputs_identical_across_tiles(gpu, shape, limbs, range_frac):
    """Static-range epilogue: limb-plane output (next conv's input), limb-plane residual, overflow
    flag and fp32 output agree bitwise across every tile config, and the
    emitted digits are clamp(rne(y * QMAX / range))."""
    from smpq import ops
    cin, cout, k, s, h = shape
    wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin + 5 * cout)
    g = torch.Generator().manual_seed(11)
    x = torch.relu(torch.randn(3, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    ho = (h + 2 * (k // 2) - k) // s + 1
    rq = ops.act_quantize(torch.randn(3, ho, ho, cout, generator=g).clamp(-4, 4).to(gpu),
                          torch.full((3,), 4.0, device=gpu), limbs)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=True,
                       residual_q=rq, residual_range=4.0)
    rng = float(ref.abs().max()) * range_frac
    outs = []
    for c in ops.tile_configs():
        if not ops._tile_fits(c, limbs, 1, cout, cin, k) or ops.tile_kind(c) in _LEAN_ONLY:
            continue
        ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
        y, yq = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=True, tile_cfg=c,
                             emit_range=rng, overflow=ovf, want_f32=True, residual_q=rq, residual_range=4.0)
        outs.append((c, y, yq, ovf))
    assert any(ops.tile_kind(c) == ops.TILE_LDS_DMA for c, *_ in outs)
    c0, y0, yq0, ovf0 = outs[0]
    assert torch.equal(y0, ref)
    for c, y, yq, ovf in outs[1:]:
        assert torch.equal(y, y0), c
        assert torch.equal(yq, yq0), c
        assert torch.equal(ovf, ovf0), c
    qmax = LIMB_QMAX[limbs]
    inv = np.float32(qmax) / np.float32(rng)  # the kernel's yq_inv, in float32 like the C side
    qf = np.rint(y0.cpu().numpy().astype(np.float32) * inv)
    q = sum(yq0[l].cpu().numpy().astype(np.int64) * 256 ** l for l in range(limbs))
    assert (yq0.cpu().numpy().astype(np.int64) >= -128).all()
    np.testing.assert_array_equal(q, np.clip(qf, -qmax, qmax).astype(np.int64))
    assert int(ovf0.item()) == int((np.abs(qf) > qmax).any())
    assert int(ovf0.item()) == (1 if range_frac < 1 else 0)


@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("range_frac", [2.0, 0.5])
@pytest.mark.parametrize("limbs", [2, 3])
@pytest.mark.parametrize("shape", [(64, 256, 1, 1, 20), (128, 64, 3, 2, 17), (64, 80, 3, 1, 9), (256, 128, 1, 1, 12)],
                         ids=lambda s: "c%d_o%d_k%d_s%d_h%d" % s)
def test_lean_static_epilogue(gpu, shape, limbs, range_frac, relu):
    """The lean static epilogue (limb planes only: the engine's block-internal convs) folds 1/step
    into the column scale: its codes agree bitwise across every tile config, are within one code
    of clamp(rne(y * QMAX / range)) of the general epilogue's fp32 y (and equal almost always),
    and it raises the overflow flag exactly when the general epilogue does."""
    from smpq import ops
    cin, cout, k, s, h = shape
    wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin + 7 * cout)
    g = torch.Generator().manual_seed(12)
    x = torch.relu(torch.randn(3, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    ho = (h + 2 * (k // 2) - k) // s + 1
    rq = ops.act_quantize(torch.randn(3, ho, ho, cout, generator=g).clamp(-4, 4).to(gpu),
                          torch.full((3,), 4.0, device=gpu), limbs)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    kw = dict(relu=relu, residual_q=rq, residual_range=4.0)
    ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, **kw)
    rng = float(ref.abs().max()) * range_frac
    outs = []
    for c in ops.tile_configs():
        if not ops._tile_fits(c, limbs, 1, cout, cin, k) or ops.tile_kind(c) not in (ops.TILE_LDS_DMA,
                                                                                            ops.TILE_LDS_DMA_K128):
            continue
        ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
        y, yq = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, tile_cfg=c,
                             emit_range=rng, overflow=ovf, want_f32=False, **kw)
        assert y is None
        outs.append((c, yq, ovf))
    c0, yq0, ovf0 = outs[0]
    for c, yq, ovf in outs[1:]:
        assert torch.equal(yq, yq0), c
        assert torch.equal(ovf, ovf0), c
    ovf_full = torch.zeros(1, dtype=torch.int32, device=gpu)
    yf, yqf = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, tile_cfg=outs[0][0],
                           emit_range=rng, overflow=ovf_full, want_f32=True, **kw)
    assert torch.equal(yf, ref)
    lean = sum(yq0[l].cpu().numpy().astype(np.int64) * 256 ** l for l in range(limbs))
    full = sum(yqf[l].cpu().numpy().astype(np.int64) * 256 ** l for l in range(limbs))
    # at 24 bits a code unit is about one fp32 ulp of z, so the two formulas' roundings differ in
    # the last code unit or two (1.2e-7 of the range); at 16 bits almost never
    diff = np.abs(lean - full)
    assert diff.max() <= (1 if limbs == 2 else 2)
    if limbs == 2:
        assert (diff != 0).mean() < 0.01
    if relu:
        assert lean.min() >= 0
    assert int(ovf0.item()) == int(ovf_full.item()) == (1 if range_frac < 1 else 0)


def test_conv_rejects_unsupported_geometry(gpu):
    """cout % 16 != 0 (the reference's ResNets never have it) is refused with a clean error by the
    C-ABI, before any launch; QConv2d sends such a conv to torch (stats['fp32_conv'])."""
    from smpq import _lib, ops
    from smpq.qconv import QConv2d
    wd, step, codes, offset = make_layer(gpu, 64, 100, 3, seed=5)
    x = torch.randn(1, 6, 6, 64, generator=torch.Generator().manual_seed(6)).to(gpu)
    am = ops.act_absmax(x)
    with pytest.raises((ValueError, _lib.SmpqError), match="multiple of 16"):
        ops.conv2d_q(ops.act_quantize(x, am, 3), am, codes, offset, 3, 3, 1, 1, step, torch.zeros(100, device=gpu))
    assert not QConv2d(64, 100, 3, padding=1).to(gpu).hip_supported()


def test_conv_offsets_exercised(gpu):
    # 8-bit channels need a code offset whenever their code range is not inside [-128, 127]
    off = run_conv_case(gpu, 256, 256, 1, 1, 14, limbs=2, seed=3)
    assert (off != 0).any()


# ----------------------------------------------------------------------------------------------
def _golden():
    return np.load(os.path.join(GOLDEN, "model_goldens.npz"), allow_pickle=False)


def build_model(gpu, arch, assign, cal_case=None):
    import resnet
    from smpq import assignments
    torch.manual_seed(0)
    net = getattr(resnet, arch)()
    if cal_case is not None:
        g = _golden()
        sd = net.state_dict()
        pref = cal_case + "/bn/"
        for k in g.files:
            if k.startswith(pref):
                sd[k[len(pref):]].copy_(torch.from_numpy(g[k]))
    net = net.to(gpu).eval()
    if assign:
        # the goldens are the reference run on the CPU: quantize with torch-CPU rounding
        assignments.apply_assignment(net, assign, semantics="cpu")
    return net


@pytest.mark.parametrize("mode", ["static", "dynamic"])
@pytest.mark.parametrize("limbs", [2, 3])
@pytest.mark.parametrize("case,arch,assign,batch", [
    ("r18_u8", "resnet18", "r18_u8", 2), ("r18_u8_b1", "resnet18", "r18_u8", 1), ("r50_mixed", "resnet50", "r50_mixed", 2),
    ("r34_4bit", "resnet34", "r34_4bit", 2), ("r18_u8_cal", "resnet18", "r18_u8", 16),
    ("r50_mixed_cal", "resnet50", "r50_mixed", 8)])
def test_model_logits_vs_reference(gpu, case, arch, assign, batch, limbs, mode):
    from smpq import engine, ops, stats
    g = _golden()
    net = build_model(gpu, arch, assign, case if case.endswith("_cal") else None)
    for k in g.files:  # fake-quantized weights identical to the reference's (checksums)
        if k.startswith(case + "/qsum/"):
            w = net.state_dict()[k[len(case + "/qsum/"):]].double().cpu()
            np.testing.assert_allclose([w.sum().item(), w.abs().sum().item()], g[k], rtol=1e-12, atol=1e-12)
    x = torch.randn(batch, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    old_limbs = ops.get_act_limbs()
    ops.set_act_limbs(limbs)
    engine.set_range_mode(mode)
    engine.USE_GRAPH[0] = False  # count launches of one eager forward (graphs: test_graph_replay_*)
    try:
        xg = x.to(gpu)
        with torch.no_grad():
            if mode == "static":
                net(xg)  # calibration forward (dynamic ranges)
            c0 = stats["calibrations"]
            before = stats["hip_conv"]
            y = net(xg).double().cpu().numpy()
            if mode == "static":
                assert stats["calibrations"] == c0  # this forward ran on the static ranges
        nq = {"resnet18": 16 + 1 + 3, "resnet34": 32 + 1 + 3, "resnet50": 48 + 1 + 4}[arch]
        # static mode runs the batch as engine.STREAMS slices (one launch per conv per slice)
        slices = engine.STREAMS[0] if (mode == "static" and xg.shape[0] >= 2 * engine.STREAMS[0]) else 1
        assert stats["hip_conv"] - before == nq * slices  # every conv incl. stem + downsample on HIP
    finally:
        ops.set_act_limbs(old_limbs)
        engine.set_range_mode("static")
        engine.USE_GRAPH[0] = True
    ref = g[case + "/logits"].astype(np.float64)
    err = np.abs(y - ref).max()
    rel = err / np.abs(ref).max()
    assert rel <= LOGIT_RTOL[limbs], rel
    srt = np.sort(ref, axis=1)
    margin = srt[:, -1] - srt[:, -2]
    agree = y.argmax(1) == ref.argmax(1)
    if limbs >= 3:
        assert agree.all()  # int24 activations: top-1 identical to the reference
    else:
        # int16: identical wherever the reference's top-1 margin exceeds twice the logit error
        assert agree[margin > 2 * err].all(), (margin, agree, err)


def test_batch_invariance_and_determinism(gpu):
    """Per-image activation ranges => a quantized conv's output for an image does not depend on
    the rest of the batch (bitwise). The whole model is deterministic per batch shape; across
    batch shapes only the fp32 MIOpen stem/downsample/fc may pick other algorithms (tiny diffs)."""
    from smpq import ops
    wd, step, codes, offset = make_layer(gpu, 256, 256, 3, seed=21)
    x = torch.relu(torch.randn(256, 14, 14, 256, generator=torch.Generator().manual_seed(4))).to(gpu)
    shift = torch.zeros(256, device=gpu)

    def run(xx):
        return ops.conv2d_nhwc(xx, ops.act_absmax(xx), codes, offset, 3, 3, 1, 1, step, shift, relu=True)
    y_big = run(x)
    assert torch.equal(y_big, run(x))
    assert torch.equal(y_big[100:103], run(x[100:103].contiguous()))
    net = build_model(gpu, "resnet18", "r18_u8")
    xi = torch.randn(64, 3, 224, 224, generator=torch.Generator().manual_seed(11)).to(gpu)
    from smpq import engine
    engine.set_range_mode("dynamic")
    try:
        with torch.no_grad():
            a, b, c = net(xi), net(xi), net(xi[10:13].contiguous())
    finally:
        engine.set_range_mode("static")
    assert torch.equal(a, b)
    # every conv is on the HIP path with per-image ranges; only the fc GEMM (hipBLASLt) and the
    # avgpool reduction see the batch shape
    torch.testing.assert_close(a[10:13], c, rtol=1e-5, atol=1e-5)


def test_dropin_gpu_quantizer_and_unquantized_channels(gpu):
    import functions
    from smpq import stats
    net = build_model(gpu, "resnet18", None)
    conv = net.layer2[1].conv2
    for c in range(conv.out_channels - 1):  # leave the last channel unquantized
        functions.channel_wise_quantizationperchan(conv.weight.data, 6, c)
    assert conv._bits_host[-1] == 0 and conv.fully_quantized() is False
    x = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(2)).to(gpu)
    f0, h0 = stats["fixed_conv"], stats["hip_conv"]
    with torch.no_grad():
        net(x)
    assert stats["hip_conv"] - h0 == 20 and stats["fixed_conv"] - f0 == 20  # nothing fully quantized
    assert conv.last_path == "hip-fixed"
    functions.channel_wise_quantizationperchan(conv.weight.data, 6, conv.out_channels - 1)
    assert conv.fully_quantized()
    f0 = stats["fixed_conv"]
    with torch.no_grad():
        net(x)
    assert stats["fixed_conv"] - f0 == 19 and conv.last_path == "hip-exact8"


def test_module_path_matches_fused(gpu):
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(3)).to(gpu)
    with torch.no_grad():
        y_fused = net(x)
        net.fused = False
        y_mod = net(x)
        net.fused = True
    rel = (y_fused - y_mod).abs().max() / y_mod.abs().max()
    assert rel < 1.5e-2


def test_evaluate_acc_loss_softmax(gpu, monkeypatch):
    import functions
    monkeypatch.setenv("SMPQ_SYNTHETIC", "1")  # the synthetic loader is opt-in only
    import imagenet
    net = build_model(gpu, "resnet18", "r18_u8")
    loader = imagenet.SyntheticImageNet(n_images=8, batch_size=4)
    acc, loss, outs = functions.evaluate_acc_loss_softmax(net, gpu, loader)
    assert 0.0 <= acc <= 1.0 and np.isfinite(loss) and len(outs) == 2 and outs[0].shape == (4, 1000)
    torch.testing.assert_close(outs[0].sum(1), torch.ones(4, device=gpu))
    assert functions.KLdiv(outs, outs) == pytest.approx(0.0, abs=1e-6)


# ---- weight limbs, stem (cin = 4), pooling --------------------------------------------------
def emulate_limbs(xq_planes, wq_planes, k, stride, pad, rscale, col_scale, col_shift, residual, relu):
    """Exact emulation of conv2d_q for activation limb planes [L,n,h,w,c] and weight limb planes
    [LW,cout,kh,kw,c] (float64 GEMM of small ints is exact), with the kernel's fp32 bound."""
    n = xq_planes.shape[1]
    v = 0.0
    mag = 0.0
    smin = max(0, xq_planes.shape[0] + wq_planes.shape[0] - 4)  # kernel skips la + lw < smin
    for la in range(xq_planes.shape[0]):
        cols, ho, wo = im2col_nhwc(xq_planes[la].astype(np.float64), k, stride, pad)
        for lw in range(wq_planes.shape[0]):
            if la + lw < smin:
                continue
            t = cols @ wq_planes[lw].reshape(wq_planes.shape[1], -1).T.astype(np.float64) * 256.0 ** (la + lw)
            v = v + t
            mag = mag + np.abs(t)
    rs = np.repeat(rscale, ho * wo)[:, None]
    y = v * rs * col_scale[None, :] + col_shift[None, :]
    bound = mag * rs * np.abs(col_scale[None, :]) + np.abs(col_shift[None, :])
    if residual is not None:
        y = y + residual.reshape(y.shape)
        bound = bound + np.abs(residual.reshape(y.shape))
    if relu:
        y = np.maximum(y, 0)
    return y.reshape(n, ho, wo, -1), bound.reshape(n, ho, wo, -1)


def test_pack_weights_ex_modes(gpu):
    from smpq import ops
    g = torch.Generator().manual_seed(3)
    w = (torch.randn(70, 64, 3, 3, generator=g) * 0.05).to(gpu)
    # fixed16: unquantized weights
    codes, _, wscale, st = ops.pack_weights_ex(w, None, 2)
    assert st.cpu().tolist() == [0, 0, 70]
    m = codes[0].long() + 256 * codes[1].long()
    wk = w.permute(0, 2, 3, 1).reshape(70, -1).double()
    err = (m.double() * wscale.double()[:, None] - wk).abs()
    assert bool((err <= 0.5 * wscale.double()[:, None] * 1.005).all())
    assert int(m.abs().max()) == 32512
    codes3, _, wscale3, st3 = ops.pack_weights_ex(w, None, 3)
    assert st3.cpu().tolist() == [0, 0, 70]
    m3 = codes3[0].long() + 256 * codes3[1].long() + 65536 * codes3[2].long()
    err3 = (m3.double() * wscale3.double()[:, None] - wk).abs()
    assert bool((err3 <= 0.5 * wscale3.double()[:, None] * 1.01).all())
    assert int(m3.abs().max()) == 8323072
    # exact codes of quantized channels in two limbs
    wq = w.clone()
    step = ops.quantize_channels_(wq.reshape(70, -1), [8] * 70)
    for lw in (2, 3):
        codes2, _, wscale2, st2 = ops.pack_weights_ex(wq, step, lw)
        assert st2.cpu().tolist() == [0, 0, 0]
        m2 = sum(codes2[l].long() * 256 ** l for l in range(lw))
        # codes normalized into the top limb: wscale = step * 2^-sh, |m| << sh <= WMAX < |m| << (sh + 1)
        shift = torch.log2(step.double() / wscale2.double())
        assert torch.equal(shift, shift.round()) and int(shift.min()) >= 1
        wmax = 32512 if lw == 2 else 8323072
        top = m2.abs().amax(1)
        assert bool((top <= wmax).all()) and bool((2 * top > wmax).all())
        rec = (m2.double() * wscale2.double()[:, None]).float()
        assert torch.equal(rec.view(torch.int32), wq.permute(0, 2, 3, 1).reshape(70, -1).contiguous().view(torch.int32))


def test_mixed_exact_fixed_conv_keeps_precision(gpu):
    """A conv whose channels are partly exact 8-bit codes and partly fixed point (a mid-search
    layer) takes 24-bit weight limbs; the low-digit products its kernel skips must not cost the
    exact channels their low activation limbs (codes normalized into the top limb)."""
    from smpq import ops
    g = torch.Generator().manual_seed(77)
    cin, cout, k = 64, 32, 3
    w = (torch.randn(cout, cin, k, k, generator=g) * 0.05).to(gpu)
    wq = w.clone()
    bits = [8] * 16 + [0] * 16
    step = ops.quantize_channels_(wq.reshape(cout, -1), bits)
    codes, _, wscale, st = ops.pack_weights_ex(wq, step, 3)
    assert st.cpu().tolist() == [0, 0, 16]
    x = torch.relu(torch.randn(2, 12, 12, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    y = ops.conv2d_q(ops.act_quantize(x, am, 3), am, codes, None, k, k, 1, 1, wscale.contiguous(),
                     torch.zeros(cout, device=gpu))
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), wq.double(), padding=1).permute(0, 2, 3, 1)
    scale = ref.abs().amax()
    err_exact = ((y.double() - ref)[..., :16].abs().amax() / scale).item()
    err_fixed = ((y.double() - ref)[..., 16:].abs().amax() / scale).item()
    assert err_exact < 1e-6, err_exact  # was ~2e-3 with the codes in the low limb
    assert err_fixed < 5e-5, err_fixed  # 24-bit fixed point, skipped low-digit products


@pytest.mark.parametrize("limbs,wlimbs", [(1, 2), (2, 2), (3, 2), (3, 3)])
def test_conv_weight_limbs_vs_emulation(gpu, limbs, wlimbs):
    from smpq import ops
    g = torch.Generator().manual_seed(limbs + 40)
    cin, cout, k, s, h = 128, 96, 3, 2, 15
    w = (torch.randn(cout, cin, k, k, generator=g) * 0.05).to(gpu)
    codes, _, wscale, _ = ops.pack_weights_ex(w, None, wlimbs)
    x = torch.randn(3, h, h, cin, generator=g).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    cs = (wscale * torch.linspace(0.5, 2, cout, device=gpu)).contiguous()
    sh = torch.linspace(-1, 1, cout, device=gpu).contiguous()
    ho = (h + 2 - k) // s + 1
    res = torch.randn(3, ho, ho, cout, generator=g).to(gpu)
    outs = []
    kinds = set()
    for c in ops.tile_configs():
        if ops._tile_fits(c, limbs, wlimbs, cout, cin, k) and ops.tile_kind(c) not in _LEAN_ONLY:
            outs.append(ops.conv2d_q(xq, am, codes, None, k, k, s, 1, cs, sh, residual=res, relu=True, tile_cfg=c))
            kinds.add(ops.tile_kind(c))
    assert ops.TILE_LDS_DMA in kinds and ops.TILE_LDS_DMA_K128 in kinds
    assert len(outs) >= 1 and all(torch.equal(o, outs[0]) for o in outs)
    wq = codes.cpu().numpy().reshape(wlimbs, cout, k, k, cin)
    rscale = (am.cpu().numpy() * np.float32(1.0 / LIMB_QMAX[limbs])).astype(np.float64)
    ye, bound = emulate_limbs(xq.cpu().numpy(), wq, k, s, 1, rscale, cs.cpu().numpy().astype(np.float64),
                              sh.cpu().numpy().astype(np.float64), res.cpu().numpy().astype(np.float64), True)
    err = np.abs(outs[0].cpu().numpy() - ye)
    assert (err <= 2e-6 * bound + 1e-30).all()


def s2d_to_image_planes(xs):
    """Space-to-depth planes [L, n, h2, w2, 16] -> the 4-channel image planes [L, n, 2 h2, 2 w2, 4]
    they hold (channel (dy*2 + dx)*4 + c = pixel (2i + dy, 2j + dx), channel c)."""
    L, n, h2, w2, _ = xs.shape
    return xs.reshape(L, n, h2, w2, 2, 2, 4).transpose(0, 1, 2, 4, 3, 5, 6).reshape(L, n, 2 * h2, 2 * w2, 4)


def s2d_codes_to_7x7(codes16):
    """s2d stem codes [LW, cout, 256] (K order [ty][tx][dy][dx][ci], original tap
    (2 ty + dy - 1, 2 tx + dx - 1)) -> [LW, cout, 7, 7, 4]; the taps outside 7x7 must be zero."""
    lw, cout, _ = codes16.shape
    c = codes16.reshape(lw, cout, 4, 4, 2, 2, 4).astype(np.int64)
    out = np.zeros((lw, cout, 8, 8, 4), np.int64)  # kernel rows / cols -1 .. 6 at index +1
    for ty in range(4):
        for tx in range(4):
            for dy in range(2):
                for dx in range(2):
                    out[:, :, 2 * ty + dy, 2 * tx + dx] = c[:, :, ty, tx, dy, dx]
    assert not out[:, :, 0].any() and not out[:, :, :, 0].any()
    return out[:, :, 1:, 1:]


@pytest.mark.parametrize("limbs", [2, 3])
@pytest.mark.parametrize("hw", [(40, 36), (37, 41), (224, 224), (33, 2)])
def test_image_quantize_s2d_and_stem_conv(gpu, limbs, hw):
    """The space-to-depth stem (the only stem path since ABI 4): the image quantizer's digits (even
    and odd sizes: an odd h / w gets a zero row / column), the conv against an exact emulation of
    the 7x7/2/3 conv on the quantized image, bitwise identical across every tile config (fp32 and
    limb-plane outputs), and within the activation quantization bound of the fp64 conv."""
    from smpq import _lib, ops
    g = torch.Generator().manual_seed(8 + limbs + hw[0])
    h, w = hw
    x = torch.randn(2, 3, h, w, generator=g).to(gpu)
    x[1] *= 3
    am = ops.act_absmax(x)
    xs = ops.image_quantize_s2d(x, am, limbs)
    assert xs.shape == (limbs, 2, (h + 1) // 2, (w + 1) // 2, 16)
    img = s2d_to_image_planes(xs.cpu().numpy())
    q = sum(img[l].astype(np.int64) * 256 ** l for l in range(limbs))
    qmax = np.float32(LIMB_QMAX[limbs])
    inv = (qmax / am.cpu().numpy()).astype(np.float32)
    exp = np.rint((x.permute(0, 2, 3, 1).cpu().numpy() * inv[:, None, None, None]).astype(np.float32))
    np.testing.assert_array_equal(q[:, :h, :w, :3], exp.astype(np.int64))
    assert not q[..., 3].any() and not q[:, h:].any() and not q[:, :, w:].any()
    wt = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(gpu)
    lw = max(2, limbs)
    codes16, wscale = ops.pack_weights_s2d(wt, lw)
    cs = (wscale * torch.linspace(0.5, 2, 64, device=gpu)).contiguous()
    sh = torch.linspace(-1, 1, 64, device=gpu).contiguous()
    outs = []
    for c in ops.tile_configs():
        ya = torch.zeros(2, device=gpu)
        try:
            y = ops.stem_conv_s2d(xs, am, codes16, h, w, cs, sh, relu=True, y_absmax=ya, tile_cfg=c)
        except _lib.SmpqError:
            continue  # not built for the stem (64 output channels per block only)
        outs.append((c, y, ya))
    assert len(outs) >= 3
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    y0 = outs[0][1]
    assert y0.shape == (2, ho, wo, 64)
    for c, y, ya in outs[1:]:
        assert torch.equal(y, y0), c
        assert torch.equal(ya, outs[0][2]), c
    rscale = (am.cpu().numpy() * np.float32(1.0 / LIMB_QMAX[limbs])).astype(np.float64)
    ye, bound = emulate_limbs(img, s2d_codes_to_7x7(codes16.cpu().numpy()), 7, 2, 3, rscale,
                              cs.cpu().numpy().astype(np.float64), sh.cpu().numpy().astype(np.float64), None, True)
    assert ye.shape == y0.shape
    assert (np.abs(y0.cpu().numpy() - ye) <= 2e-6 * bound + 1e-30).all()
    np.testing.assert_array_equal(outs[0][2].cpu().numpy(), np.abs(y0.cpu().numpy()).reshape(2, -1).max(1))
    ref = torch.nn.functional.conv2d(x.double(), wt.double(), stride=2, padding=3)
    ref = torch.relu(ref * (cs / wscale).double()[None, :, None, None] + sh.double()[None, :, None, None])
    ref = ref.permute(0, 2, 3, 1).cpu().numpy()
    assert np.abs(y0.cpu().numpy() - ref).max() <= 2e-3 * np.abs(ref).max()
    # limb-plane output (lean static epilogue): identical across tiles, within a code unit or two of
    # rne(y * QMAX / range) of the fp32 output
    rng = float(y0.abs().max()) * 1.5
    yq0 = None
    for c, _, _ in outs:
        ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
        _, yq = ops.stem_conv_s2d(xs, am, codes16, h, w, cs, sh, relu=True, tile_cfg=c, emit_range=rng,
                                  overflow=ovf, want_f32=False)
        yq0 = yq if yq0 is None else yq0
        assert torch.equal(yq, yq0), c
        assert int(ovf.item()) == 0
    lean = sum(yq0[l].cpu().numpy().astype(np.int64) * 256 ** l for l in range(limbs))
    full = np.rint(y0.cpu().numpy() * (qmax / np.float32(rng))).astype(np.int64)
    assert np.abs(lean - full).max() <= (1 if limbs == 2 else 2)


@pytest.mark.parametrize("hw", [(224, 224), (225, 223)])
def test_module_path_stem_is_the_s2d_kernel(gpu, hw):
    """QConv2d.forward of the stem (the module path the unfused forward and a user's own
    call take) runs the space-to-depth kernel: bitwise the same as stem_conv_s2d on the packed
    codes, within the activation-quantization bound of the fp64 conv, odd sizes included."""
    from smpq import ops
    net = build_model(gpu, "resnet18", None)
    conv = net.conv1
    h, w = hw
    x = torch.randn(2, 3, h, w, generator=torch.Generator().manual_seed(41)).to(gpu)
    with torch.no_grad():
        y = conv(x)
    assert conv.last_path == "hip-fixed-s2d" and y.shape == (2, 64, (h + 1) // 2, (w + 1) // 2)
    codes, wscale, _ = conv.packed_s2d()
    am = ops.act_absmax(x)
    ref = ops.stem_conv_s2d(ops.image_quantize_s2d(x, am), am, codes, h, w, wscale.contiguous(),
                            torch.zeros(64, device=gpu), relu=False)
    assert torch.equal(y, ref.permute(0, 3, 1, 2))
    f64 = torch.nn.functional.conv2d(x.double(), conv.weight.double(), stride=2, padding=3)
    bound = 0.5 * (am.double() / LIMB_QMAX[3])[:, None, None, None] * \
        torch.nn.functional.conv2d(torch.ones_like(x).double(), conv.weight.double().abs(), stride=2, padding=3)
    assert bool(((y.double() - f64).abs() <= bound * 1.01 + 1e-6 * f64.abs().max()).all())


def test_quantized_stem_channels_exact(gpu):
    """A stem with quantized channels (channel_wise_quantizationperchan on conv1's weight) runs on
    the s2d kernel with those channels' exact codes (pack_weights_s2d with the recorded steps): its
    output equals the fp64 conv of the quantized weights on the quantized image."""
    from smpq import ops
    g = torch.Generator().manual_seed(19)
    wt = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(gpu)
    step = ops.quantize_channels_(wt.reshape(64, -1), [8] * 32 + [0] * 32)
    for lw in (2, 3):
        codes16, wscale = ops.pack_weights_s2d(wt, lw, step=step)
        m = s2d_codes_to_7x7(codes16.cpu().numpy())
        val = sum(m[l] * 256 ** l for l in range(lw))  # [cout, 7, 7, 4]
        rec = (val[..., :3].transpose(0, 3, 1, 2) * wscale.cpu().numpy().astype(np.float64)[:, None, None, None])
        # quantized channels: exact codes (m * 2^-sh * step reproduces the weight bit for bit)
        np.testing.assert_array_equal(rec[:32].astype(np.float32), wt[:32].cpu().numpy())
        assert np.abs(rec[32:] - wt[32:].cpu().numpy()).max() <= 0.5 * wscale[32:].max().item() * 1.01


@pytest.mark.parametrize("limbs", [1, 2, 3])
def test_maxpool_limbs_equals_quantized_maxpool(gpu, limbs):
    """Max pool on the codes == the codes of the max pool (monotone quantizer), bit for bit."""
    import torch.nn.functional as F
    from smpq import ops
    g = torch.Generator().manual_seed(5 + limbs)
    x = torch.relu(torch.randn(3, 17, 22, 32, generator=g)).to(gpu)  # NHWC, odd/even sizes
    rng = torch.full((3,), float(x.abs().max()) * 1.3, device=gpu)
    xq = ops.act_quantize(x, rng, limbs)
    pooled = F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1).contiguous()
    assert torch.equal(ops.maxpool_limbs(xq), ops.act_quantize(pooled, rng, limbs))


@pytest.mark.parametrize("limbs", [1, 2, 3])
@pytest.mark.parametrize("nhw", [(2, 224, 224), (3, 40, 36), (1, 32, 64), (2, 100, 220)])
def test_fused_stem_pool_bitwise(gpu, limbs, nhw):
    """conv1 + bn1 + relu + maxpool in one launch == stem_conv_s2d (static range) + maxpool_limbs,
    bit for bit: every workgroup band split (2 images -> one pooled row per band at 224; 1 image ->
    16 bands), partial column fragments (w/2 = 18, 110), negative and zero BN scales, and the
    overflow flag with a range that clamps."""
    from smpq import ops
    n, h, w = nhw
    g = torch.Generator().manual_seed(31 + limbs + h)
    wt = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(gpu)
    x = torch.randn(n, 3, h, w, generator=g).to(gpu)
    x[0] *= 3.0
    am = ops.act_absmax(x)
    lw = max(2, limbs)
    codes, wscale = ops.pack_weights_s2d(wt, lw)
    # negative scales (a BN with gamma < 0: the epilogue decreases with the conv value, so the fused
    # kernel, which pools before its epilogue, pools the minimum there) and a zero scale
    cs = (wscale * torch.linspace(-1.0, 2, 64, device=gpu)).contiguous()
    cs[5] = 0.0
    sh = torch.linspace(-1, 1, 64, device=gpu).contiguous()
    xs = ops.image_quantize_s2d(x, am, limbs)
    assert ops.stem_pool_supported(xs, codes, h, w)
    ya = torch.zeros(n, device=gpu)
    y = ops.stem_conv_s2d(xs, am, codes, h, w, cs, sh, relu=True, y_absmax=ya)
    for frac, want_ovf in ((1.5, 0), (0.3, 1)):
        rng = float(y.abs().max()) * frac
        o2 = torch.zeros(1, dtype=torch.int32, device=gpu)
        _, yq = ops.stem_conv_s2d(xs, am, codes, h, w, cs, sh, relu=True, emit_range=rng, overflow=o2,
                                  want_f32=False)
        ref = ops.maxpool_limbs(yq)
        o1 = torch.zeros(1, dtype=torch.int32, device=gpu)
        got = ops.stem_pool_s2d(xs, am, codes, h, w, cs, sh, emit_range=rng, overflow=o1)
        assert got.shape == ref.shape == (limbs, n, h // 4, w // 4, 64)
        assert torch.equal(got, ref), (frac, (got != ref).sum().item())
        assert int(o1.item()) == int(o2.item()) == want_ovf


def test_fused_stem_in_the_model(gpu):
    """The static-range forward with the fused stem gives the same logits as with the two-launch
    stem (eager and graph replay)."""
    from smpq import engine
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(17)).to(gpu)
    old = engine.FUSED_STEM[0]
    try:
        with torch.no_grad():
            engine.FUSED_STEM[0] = False
            net(x)  # calibrate
            a = net(x)
            engine.FUSED_STEM[0] = True
            b = net(x)
            c = net(x)
        assert net.conv1.last_path == "hip-fixed-s2d-pool"
    finally:
        engine.FUSED_STEM[0] = old
    assert torch.equal(a, b) and torch.equal(a, c)


@pytest.mark.parametrize("arch,assign", [("resnet50", "r50_mixed"), ("resnet18", "r18_u8")])
def test_concurrent_streams_bitwise(gpu, arch, assign):
    """The downsample branch on a side stream and the batch split into 2 / 3 slices on their own
    streams (fork/join, eager and inside the captured graph) give the same logits, bit for bit, as
    the serial forward."""
    from smpq import engine
    net = build_model(gpu, arch, assign)
    x = torch.randn(7, 3, 224, 224, generator=torch.Generator().manual_seed(23)).to(gpu)
    x2 = torch.randn(7, 3, 224, 224, generator=torch.Generator().manual_seed(24)).to(gpu)
    old = engine.CONCURRENT_DS[0], engine.USE_GRAPH[0], engine.STREAMS[0]
    got = []
    try:
        with torch.no_grad():
            engine.CONCURRENT_DS[0], engine.USE_GRAPH[0], engine.STREAMS[0] = False, False, 1
            net(x)  # calibrate
            a, a2 = net(x), net(x2)
            for streams in (1, 2, 3):
                engine.STREAMS[0] = streams
                engine.CONCURRENT_DS[0], engine.USE_GRAPH[0] = True, False
                got += [(net(x), a), (net(x2), a2)]  # eager, forked
                engine.USE_GRAPH[0] = True
                got += [(net(x), a), (net(x2), a2), (net(x), a)]  # capture, replays
    finally:
        engine.CONCURRENT_DS[0], engine.USE_GRAPH[0], engine.STREAMS[0] = old
    torch.cuda.synchronize()
    for i, (g, want) in enumerate(got):
        assert torch.equal(g, want), i


@pytest.mark.parametrize("limbs", [2, 3])
def test_maxpool_quantize(gpu, limbs):
    from smpq import ops
    x = torch.relu(torch.randn(3, 17, 18, 64, generator=torch.Generator().manual_seed(2))).to(gpu)
    am = ops.act_absmax(x)
    q, f = ops.maxpool_quantize(x, am, limbs)
    ref = torch.nn.functional.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(f, ref.contiguous())
    val = sum(q[l].long() * 256 ** l for l in range(limbs))
    qmax = np.float32(LIMB_QMAX[limbs])
    inv = (qmax / am.cpu().numpy()).astype(np.float32)
    exp = np.rint((ref.cpu().numpy() * inv[:, None, None, None]).astype(np.float32))
    np.testing.assert_array_equal(val.cpu().numpy(), exp.astype(np.int64))


def test_static_ranges_overflow_falls_back_to_dynamic(gpu):
    from smpq import engine, stats
    net = build_model(gpu, "resnet18", "r18_u8")
    x = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(12)).to(gpu)
    with torch.no_grad():
        engine.set_range_mode("dynamic")
        y_dyn = net(x)
        engine.set_range_mode("static")
        y_cal = net(x)  # calibration forward == a dynamic forward
        assert torch.equal(y_cal, y_dyn)
        y_st = net(x)
        assert (y_st - y_dyn).abs().max() <= 2e-2 * y_dyn.abs().max()
        # a 5x larger input overflows the calibrated ranges -> recomputed dynamically
        r0 = stats["overflow_reruns"]
        y_big = net(5 * x)
        assert stats["overflow_reruns"] == r0 + 1
        engine.set_range_mode("dynamic")
        y_big_dyn = net(5 * x)
        engine.set_range_mode("static")
    assert torch.equal(y_big, y_big_dyn)


@pytest.mark.parametrize("mode", ["dynamic", "static"])
def test_chunked_forward_identical(gpu, mode):
    """Infinity-Cache batch chunking changes no result (per-image independence), also with the
    chunks round-robin over 1 / 2 / 3 concurrent streams (static mode; eager and graph replay)."""
    from smpq import engine
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(12, 3, 224, 224, generator=torch.Generator().manual_seed(13)).to(gpu)
    engine.set_range_mode(mode)
    old = engine.CHUNK[0], engine.STREAMS[0], engine.USE_GRAPH[0]
    got = []
    try:
        with torch.no_grad():
            engine.set_chunk(64)
            net(x)  # calibrates in static mode
            a = net(x)
            engine.set_chunk(5)
            for streams in (1, 2, 3):
                engine.STREAMS[0] = streams
                for graph in (False, True):
                    engine.USE_GRAPH[0] = graph
                    got += [net(x), net(x)]
    finally:
        engine.set_chunk(old[0])
        engine.STREAMS[0], engine.USE_GRAPH[0] = old[1], old[2]
        engine.set_range_mode("static")
    for i, b in enumerate(got):
        assert torch.equal(a, b), i


def test_graph_replay_matches_eager(gpu):
    """Graph replay == eager, bitwise: graphs captured on the inputs' own memory (one per input
    address, no input copy) and the fallback graph that copies its input into a static buffer."""
    from smpq import engine, stats
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(14)).to(gpu)
    x2 = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(15)).to(gpu)
    old = engine.GRAPHS_PER_MODEL[0]
    try:
        with torch.no_grad():
            engine.USE_GRAPH[0] = False
            net(x)  # calibrate
            e1, e2 = net(x), net(x2)
            engine.USE_GRAPH[0] = True
            c0, r0 = stats["graph_captures"], stats["graph_replays"]
            g1 = net(x)   # capture on x's memory
            g2 = net(x2)  # capture on x2's memory
            g3 = net(x)   # replay (x's graph)
            g4 = net(x2)  # replay (x2's graph)
            x.copy_(x2)
            g5 = net(x)   # replay of x's graph on new content at the same address
            assert stats["graph_captures"] == c0 + 2 and stats["graph_replays"] == r0 + 3
            # the same address and shape in another layout (a channels_last view of x's
            # memory) must not replay x's graph, which reads its input as contiguous NCHW
            n_, c_, h_, w_ = x.shape
            xcl = x.as_strided(x.shape, (c_ * h_ * w_, 1, w_ * c_, c_))
            assert xcl.data_ptr() == x.data_ptr() and not xcl.is_contiguous()
            g6 = net(xcl)
            engine.GRAPHS_PER_MODEL[0] = 0  # fallback: one graph, inputs copied in
            net._smpq_graphs = None
            net._smpq_graph = None
            f1, f2, f3 = net(x2), net(x2.clone()), net(x2.clone())
            engine.USE_GRAPH[0] = False
            e6 = net(xcl.contiguous())
            engine.USE_GRAPH[0] = True
    finally:
        engine.GRAPHS_PER_MODEL[0] = old
        engine.USE_GRAPH[0] = True
    assert torch.equal(g1, e1) and torch.equal(g2, e2) and torch.equal(g3, e1) and torch.equal(g4, e2)
    assert torch.equal(g5, e2) and torch.equal(f1, e2) and torch.equal(f2, e2) and torch.equal(f3, e2)
    assert torch.equal(g6, e6) and not torch.equal(g6, e2)


def test_graph_fast_path_never_returns_stale_weights(gpu):
    """The replay-first fast path validates weights/BN after launching: an in-place re-quantization
    through .data (how the reference's drivers write weights) or a BN buffer change must be
    reflected in the very next call, identical to a forward with graphs disabled."""
    import functions
    from smpq import engine, stats
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(21)).to(gpu)
    engine.USE_GRAPH[0] = True
    with torch.no_grad():
        net(x)
        net(x)  # capture
        y0 = net(x)  # replay
        cal0 = stats["calibrations"]
        conv = net.layer2[1].conv2
        functions.channel_wise_quantizationperchan(conv.weight.data, 2, 3)  # in place, no _version bump
        y1 = net(x)
        assert stats["calibrations"] == cal0 + 1
        net.layer3[0].bn1.running_mean.add_(0.25)  # in-place BN buffer change
        y2 = net(x)  # the recalibration forward (dynamic ranges)
        assert stats["calibrations"] == cal0 + 2
        y3, y4 = net(x), net(x)  # recapture, replay (static ranges)
        engine.USE_GRAPH[0] = False
        e2 = net(x)  # static ranges, eager
        engine.USE_GRAPH[0] = True
    assert not torch.equal(y0, y1) and not torch.equal(y1, y2)
    assert torch.equal(y3, e2) and torch.equal(y4, e2)
    assert (y2 - e2).abs().max() <= 2e-4 * e2.abs().max()


@pytest.mark.parametrize("shape", [(64, 256, 1, 1, 20), (128, 256, 1, 1, 20), (128, 128, 3, 1, 14)],
                         ids=lambda s: "c%d_o%d_k%d_s%d_h%d" % s)
def test_tile_configs_deterministic(gpu, shape):
    """Every tile config, run repeatedly on one static-range conv with a limb-plane residual and
    both outputs, reproduces the reference config bit for bit (an intra-kernel race shows up as
    an intermittent mismatch)."""
    from smpq import ops
    cin, cout, k, s, h = shape
    limbs = 3
    wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin + 5 * cout)
    g = torch.Generator().manual_seed(11)
    x = torch.relu(torch.randn(3, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    ho = (h + 2 * (k // 2) - k) // s + 1
    rq = ops.act_quantize(torch.randn(3, ho, ho, cout, generator=g).clamp(-4, 4).to(gpu),
                          torch.full((3,), 4.0, device=gpu), limbs)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    kw = dict(residual_q=rq, residual_range=4.0, want_f32=True, relu=True)
    ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=True, residual_q=rq,
                       residual_range=4.0)
    rng = float(ref.abs().max()) * 2.0
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    y0, q0 = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, tile_cfg=1, emit_range=rng,
                          overflow=ovf, **kw)
    cfgs = [c for c in ops.tile_configs() if ops._tile_fits(c, limbs, 1, cout, cin, k)
            and ops.tile_kind(c) not in _LEAN_ONLY]  # (fp32 output + residual: not the halo kernel's)
    for c in cfgs:
        for rep in range(8):
            y, q = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, tile_cfg=c, emit_range=rng,
                                overflow=ovf, **kw)
            assert torch.equal(y, y0) and torch.equal(q, q0), (c, rep)


@pytest.mark.parametrize("shape", [(128, 256, 3, 1, 14, 1), (256, 512, 1, 2, 28, 3), (512, 128, 1, 1, 14, 1),
                                   (64, 64, 3, 1, 20, 1), (192, 80, 3, 1, 9, 1), (128, 112, 1, 1, 11, 3)],
                         ids=lambda s: "c%d_o%d_k%d_s%d_h%d_lw%d" % s)
def test_kmajor_weights_bitwise(gpu, shape):
    """The K-major weight copy (smpq_weights_kmajor, round 3) is the permutation it claims, and
    every LDS-DMA tile config reading it (smpq_conv2d_fwd_q_km) gives the row-major result bit for
    bit — fp32 output, limb planes, limb-plane residual, overflow flag — incl. partial channel
    tiles (cout % BC != 0), 128-B K steps and 24-bit fixed-point weights."""
    from smpq import ops
    cin, cout, k, s, h, wl = shape
    limbs = 3
    g = torch.Generator().manual_seed(cin * 7 + cout)
    w = (torch.randn(cout, cin, k, k, generator=g) * 0.05).to(gpu)
    if wl == 1:
        step = ops.quantize_channels_(w.reshape(cout, -1), [6] * cout)
        codes, offset, wscale, st = ops.pack_weights_ex(w, step, 1)
        offset = offset if bool((offset != 0).any()) else None
    else:
        codes, _, wscale, st = ops.pack_weights_ex(w, None, wl)
        offset = None
    km = codes._smpq_km
    K = codes.shape[-1]
    assert torch.equal(km, codes.view(wl, cout, K // 64, 64).permute(0, 2, 1, 3).contiguous())
    x = torch.relu(torch.randn(3, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    ho = (h + 2 * (k // 2) - k) // s + 1
    rq = ops.act_quantize(torch.randn(3, ho, ho, cout, generator=g).clamp(-4, 4).to(gpu),
                          torch.full((3,), 4.0, device=gpu), limbs)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    kw = dict(residual_q=rq, residual_range=4.0, want_f32=True, relu=True)
    ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, wscale, shift, weight_layout="rowmajor", **kw)
    rng = float(ref.abs().max()) * 2.0
    cfgs = [c for c in ops.tile_configs() if ops.tile_kind(c) in (ops.TILE_LDS_DMA, ops.TILE_LDS_DMA_K128)
            and ops._tile_fits(c, limbs, wl, cout, cin, k)]
    assert cfgs
    for c in cfgs:
        o0 = torch.zeros(1, dtype=torch.int32, device=gpu)
        o1 = torch.zeros(1, dtype=torch.int32, device=gpu)
        y0, q0 = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, wscale, shift, tile_cfg=c, emit_range=rng,
                              overflow=o0, weight_layout="rowmajor", **kw)
        y1, q1 = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, wscale, shift, tile_cfg=c, emit_range=rng,
                              overflow=o1, **kw)
        assert torch.equal(y0, y1) and torch.equal(q0, q1) and torch.equal(o0, o1), c
        assert torch.equal(y0, ref), c


def test_forward_independent_of_previous_input(gpu):
    """A forward's result must not depend on what ran before it (stale memory or registers): the
    static-range forward of x, then of x2, then of x again gives x's logits bit for bit, several
    times over (a VMEM store-data hazard once left x2's limb-plane bytes in x's activations)."""
    from smpq import engine
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(14)).to(gpu)
    x2 = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(15)).to(gpu)
    use = engine.USE_GRAPH[0]
    engine.USE_GRAPH[0] = False
    try:
        with torch.no_grad():
            net(x)
            e1 = net(x)
            for _ in range(3):
                net(x2)
                assert torch.equal(net(x), e1)
    finally:
        engine.USE_GRAPH[0] = use


def _fresh_dynamic_logits(gpu, net, x):
    """Logits of a freshly built model holding net's current state (dynamic ranges, no caches)."""
    import resnet
    from smpq import checkpoint, engine
    fresh = getattr(resnet, "resnet50")().to(gpu).eval()
    fresh.load_state_dict(net.state_dict())
    for a, b in zip(net.modules(), fresh.modules()):
        if hasattr(a, "_bits_host"):
            b._bits_host = a._bits_host.copy()
            b._meta_gen += 1
    prev = engine.get_range_mode()
    engine.set_range_mode("dynamic")
    try:
        with torch.no_grad():
            return fresh(x)
    finally:
        engine.set_range_mode(prev)


@pytest.mark.parametrize("mode", ["static", "dynamic"])
def test_cache_sees_every_kind_of_weight_change(gpu, mode):
    """the cached forward (packed codes, folded BN, ranges, HIP graph) must never return
    stale logits — not after a replaced Parameter, load_state_dict(assign=True), a swapped
    submodule, or writes through .data that leave _version unchanged (caught by the device
    fingerprint)."""
    import functions
    from smpq import engine, stats
    from smpq.qconv import QConv2d
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(31)).to(gpu)
    engine.set_range_mode(mode)
    engine.USE_GRAPH[0] = True
    tol = 2e-4 if mode == "static" else 0.0

    def fwd():
        with torch.no_grad():
            net(x)
            return net(x)  # static: capture / replay path after a change

    def check(tag):
        y = fwd()
        ref = _fresh_dynamic_logits(gpu, net, x)
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        assert err <= tol, (tag, err)
        return y

    try:
        y_prev = check("start")
        conv = net.layer1[1].conv2
        # 1. raw .data write of one channel, bypassing the drop-in quantizer (no _version bump)
        r0 = stats["stale_reruns"]
        w = conv.weight.data
        w[5] = functions.quantize_wgt(w[5].clone(), 4)
        y = check("data-write")
        assert stats["stale_reruns"] > r0 and not torch.equal(y, y_prev)
        y_prev = y
        # 2. .data.copy_ of a whole weight
        conv3 = net.layer3[2].conv3
        conv3.weight.data.copy_(conv3.weight.data * 0.5)
        y = check("data-copy")
        assert not torch.equal(y, y_prev)
        y_prev = y
        # 3. BN buffer through .data
        net.layer2[0].bn2.running_var.data.mul_(4.0)
        y = check("bn-data")
        assert not torch.equal(y, y_prev)
        y_prev = y
        # 4. a replaced Parameter (new tensor object)
        c = net.layer4[0].conv1
        c.weight = torch.nn.Parameter(c.weight.detach().clone() * 1.5)
        y = check("param-replace")
        assert not torch.equal(y, y_prev)
        y_prev = y
        # 5. load_state_dict(assign=True)
        sd = {k: v.clone() for k, v in net.state_dict().items()}
        sd["layer2.1.conv1.weight"] = sd["layer2.1.conv1.weight"] * 0.75
        net.load_state_dict(sd, assign=True)
        y = check("assign")
        assert not torch.equal(y, y_prev)
        y_prev = y
        # 6. a swapped submodule
        old = net.layer3[1].conv2
        new = QConv2d(old.in_channels, old.out_channels, 3, padding=1, bias=False).to(gpu)
        with torch.no_grad():
            new.weight.copy_(old.weight * -1.0)
        net.layer3[1].conv2 = new
        y = check("swap")
        assert not torch.equal(y, y_prev)
    finally:
        engine.set_range_mode("static")


def test_device_fingerprint_matches_host(gpu):
    from smpq.fingerprint import Fingerprinter, host_fingerprint
    g = torch.Generator().manual_seed(9)
    ts = [torch.randn(n, generator=g) for n in (16, 70000, 16384, 5)] + [torch.randint(-128, 127, (64,), dtype=torch.int8)]
    fp = Fingerprinter([t.to(gpu) for t in ts], gpu)
    got = fp.ref.cpu().numpy().view(np.uint64).tolist()
    assert got == [host_fingerprint(t) for t in ts]
    flag = torch.zeros(1, dtype=torch.int32, device=gpu)
    fp.check(flag)
    assert int(flag.item()) == 0
    fp.tensors[1][12345] += 1.0
    fp.check(flag)
    assert int(flag.item()) == 1


# per-image bound: max_c |logit - ref| / max_c |ref| of every single image
PER_IMAGE_RTOL = 2e-4


@pytest.mark.parametrize("case,arch,assign,batch", [
    ("r50_mixed_cal", "resnet50", "r50_mixed", 256),   # BASELINE.json configs[2] (the bench)
    ("r18_u8_cal", "resnet18", "r18_u8", 256),         # configs[1]
    ("r34_4bit_cal", "resnet34", "r34_4bit", 512)])    # configs[4]
def test_bench_workload_parity_full_size(gpu, case, arch, assign, batch):
    """Parity at the bench configs' full sizes: the production path (L=3, static ranges calibrated
    on a first batch, HIP graph, two stream slices) on the BN-recalibrated parity model vs the
    reference's CPU forward restated in oracle/torch_ref.py (the same torch-CPU operators; pinned
    against the reference's own logits by test_oracle_golden) on the same fake-quantized weights
    and the same images. Stated tolerance: max |logit - ref| <= 2e-4 max |ref| over
    the batch, <= PER_IMAGE_RTOL of each image's own max |ref|, and top-1 identical for every image
    (north star: top-1 within +-0.05 %, i.e. no flip at these batch sizes)."""
    from oracle import torch_ref
    from smpq import engine, ops, stats
    old = ops.get_act_limbs(), engine.get_range_mode()
    ops.set_act_limbs(3)  # the bench's parity mode
    engine.set_range_mode("static")
    try:
        net = build_model(gpu, arch, assign, case)
        sd = {k: v.detach().cpu() for k, v in net.state_dict().items() if not k.endswith(("qbits", "qstep"))}
        x_cal = torch.randn(batch, 3, 224, 224, generator=torch.Generator().manual_seed(2023))
        x = torch.randn(batch, 3, 224, 224, generator=torch.Generator().manual_seed(2024))
        with torch.no_grad():
            net(x_cal.to(gpu))  # calibration on another batch, as an evaluation loop does
            c0 = stats["calibrations"] + stats["overflow_reruns"]
            net(x.to(gpu))  # graph capture
            y = net(x.to(gpu)).double().cpu()  # graph replay: the bench's timed path
            reruns = stats["calibrations"] + stats["overflow_reruns"] - c0
    finally:
        ops.set_act_limbs(old[0])
        engine.set_range_mode(old[1])
    ref = torch_ref.resnet_forward(arch, sd, x).double()
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    per_img = ((y - ref).abs().amax(1) / ref.abs().amax(1)).max().item()
    agree = (y.argmax(1) == ref.argmax(1)).double().mean().item()
    top2 = ref.topk(2, dim=1).values
    print("full-size parity %s B=%d: max rel logit err %.2e, worst per-image rel err %.2e, top-1 agreement "
          "%d/%d, smallest reference top-1 margin %.3e, recalibrations %d"
          % (case, batch, err, per_img, int(round(agree * batch)), batch,
             (top2[:, 0] - top2[:, 1]).min().item(), reruns))
    assert err <= 2e-4, err
    assert per_img <= PER_IMAGE_RTOL, per_img
    assert torch.equal(y.argmax(1), ref.argmax(1)), agree


@pytest.mark.parametrize("arch,assign", [("resnet50", "r50_mixed"), ("resnet18", "r18_u8")])
def test_check_stream_fork_capture_replay(gpu, arch, assign):
    """Verdict r5 item 2: the capture topology of commit a082ca2 — the weights' content check on a
    stream forked from the capture stream only for it, beside the downsample side-stream forks
    (STREAMS 1) or the batch-slice forks (STREAMS 2, 3), joined before EndCapture — which crashed
    one CUDAGraph.replay() in round 5's GPU suite. Every fork is one level deep (the topology ROCm
    7.2 captures: tools/repro_graph_fork.py); captured and replayed here in the test's call order,
    bitwise equal to the serial eager forward."""
    from smpq import engine
    net = build_model(gpu, arch, assign)
    x = torch.randn(7, 3, 224, 224, generator=torch.Generator().manual_seed(23)).to(gpu)
    x2 = torch.randn(7, 3, 224, 224, generator=torch.Generator().manual_seed(24)).to(gpu)
    shipped = engine._capture_locked

    def capture_with_check_stream(model, x_in, cal):
        g = torch.cuda.CUDAGraph()
        ctx = engine.Ctx(x_in.shape[0], x_in.device, ranges=cal[0], cache=cal[2])
        pool = getattr(model, "_smpq_pool", None)
        if pool is None or pool[0] != x_in.device:
            pool = model._smpq_pool = (x_in.device, torch.cuda.graph_pool_handle())
        torch.cuda.synchronize()
        with torch.cuda.graph(g, pool=pool[1], capture_error_mode="thread_local"):
            ctx.overflow = torch.zeros(2, dtype=torch.int32, device=x_in.device)
            main = torch.cuda.current_stream()
            chk = engine._stream((x_in.device, "check"))
            chk.wait_stream(main)
            with torch.cuda.stream(chk):
                cal[3].check(ctx.overflow[1:])
            y_static = engine._forward(model, x_in, ctx)
            main.wait_stream(chk)
        engine.stats["graph_captures"] += 1
        return g, ctx, y_static

    old = engine.CONCURRENT_DS[0], engine.USE_GRAPH[0], engine.STREAMS[0]
    got = []
    try:
        engine._capture_locked = capture_with_check_stream
        with torch.no_grad():
            engine.CONCURRENT_DS[0], engine.USE_GRAPH[0], engine.STREAMS[0] = False, False, 1
            net(x)  # calibrate
            a, a2 = net(x), net(x2)
            for streams in (1, 2, 3):
                engine.STREAMS[0], engine.CONCURRENT_DS[0], engine.USE_GRAPH[0] = streams, True, True
                got += [(net(x), a), (net(x2), a2), (net(x), a), (net(x2), a2)]  # 2 captures, 2 replays
    finally:
        engine._capture_locked = shipped
        engine.CONCURRENT_DS[0], engine.USE_GRAPH[0], engine.STREAMS[0] = old
    torch.cuda.synchronize()
    for i, (g, want) in enumerate(got):
        assert torch.equal(g, want), i
