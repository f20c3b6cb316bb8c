"""Persistent-block tiles of the LDS-DMA conv kernel (conv_glds_kernel.h kGldsP, C-ABI numbers
after the halo tiles): a block runs several tiles and issues the next tile's first K steps before
this tile's epilogue. Every output mode must equal the plain tiles' bit for bit — at sizes where
the whole-GPU variants (as many blocks as fit at once) really give blocks several tiles, with a
partial last round of tiles, partial channel tiles, limb-plane residuals, fp32 residuals, per-image
maxima, overflow flags and 24-bit fixed-point (3-limb) weights. Every call goes through the C-ABI."""
import pytest
import torch

from test_gpu import make_layer

pytestmark = pytest.mark.gpu


def _persistent_cfgs(ops, limbs, wlimbs, cout, cin, k):
    """The persistent-block tiles that take this conv: the C-ABI numbers after the last halo tile."""
    last_halo = max(c for c in ops.tile_configs() if ops.tile_kind(c) == ops.TILE_HALO3X3)
    return [c for c in ops.tile_configs() if c > last_halo and ops._tile_fits(c, limbs, wlimbs, cout, cin, k)]


def _plain_cfgs(ops, limbs, wlimbs, cout, cin, k):
    last = min(c for c in ops.tile_configs() if ops.tile_kind(c) == ops.TILE_HALO3X3)
    return [c for c in ops.tile_configs() if c < last and ops._tile_fits(c, limbs, wlimbs, cout, cin, k)]


@pytest.mark.parametrize("shape", [(64, 256, 1, 1, 56, 16), (1024, 256, 1, 1, 14, 128), (256, 1024, 1, 1, 14, 64),
                                   (2048, 512, 1, 1, 7, 256), (128, 112, 1, 1, 11, 40), (64, 64, 3, 1, 28, 16)],
                         ids=lambda s: "c%d_o%d_k%d_s%d_h%d_n%d" % s)
def test_persistent_lean_residual_bitwise(gpu, shape):
    """The block convs' lean epilogues (ReLU + limb-plane residual, and ReLU alone) and the overflow
    flag, in range and overflowing, against the plain tiles."""
    from smpq import ops
    cin, cout, k, s, h, n = shape
    limbs = 3
    wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin + cout + n)
    g = torch.Generator().manual_seed(h + n)
    x = torch.relu(torch.randn(n, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    ho = (h + 2 * (k // 2) - k) // s + 1
    rq = ops.act_quantize(torch.randn(n, ho, ho, cout, generator=g).clamp(-4, 4).to(gpu),
                          torch.full((n,), 4.0, device=gpu), limbs)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    pers = _persistent_cfgs(ops, limbs, 1, cout, cin, k)
    assert pers
    base = _plain_cfgs(ops, limbs, 1, cout, cin, k)[0]
    for resid in (True, False):
        kw = dict(relu=True, residual_q=rq, residual_range=4.0) if resid else dict(relu=True)
        ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, tile_cfg=base, **kw)
        for frac in (2.0, 0.5):
            rng = float(ref.abs().max()) * frac
            o0 = torch.zeros(1, dtype=torch.int32, device=gpu)
            _, q0 = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, tile_cfg=base, emit_range=rng,
                                 overflow=o0, want_f32=False, **kw)
            assert int(o0.item()) == (1 if frac < 1 else 0)
            for c in pers:
                o = torch.zeros(1, dtype=torch.int32, device=gpu)
                _, q = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, tile_cfg=c, emit_range=rng,
                                    overflow=o, want_f32=False, **kw)
                assert torch.equal(q, q0), (c, resid, frac)
                assert torch.equal(o, o0), (c, resid, frac)


@pytest.mark.parametrize("shape", [(256, 512, 1, 2, 28, 64), (1024, 2048, 1, 2, 14, 64), (64, 256, 1, 1, 56, 16)],
                         ids=lambda s: "c%d_o%d_k%d_s%d_h%d_n%d" % s)
def test_persistent_downsample_bitwise(gpu, shape):
    """The downsample convs: 24-bit fixed-point weights (3 weight limbs), no ReLU, no residual."""
    from smpq import ops
    cin, cout, k, s, h, n = shape
    limbs, wl = 3, 3
    g = torch.Generator().manual_seed(cin + cout)
    w = (torch.randn(cout, cin, k, k, generator=g) * 0.05).to(gpu)
    codes, _, wscale, _ = ops.pack_weights_ex(w, None, wl)
    x = torch.relu(torch.randn(n, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    pers = _persistent_cfgs(ops, limbs, wl, cout, cin, k)
    assert pers
    base = _plain_cfgs(ops, limbs, wl, cout, cin, k)[0]
    ref = ops.conv2d_q(xq, am, codes, None, k, k, s, 0, wscale, shift, tile_cfg=base)
    rng = float(ref.abs().max()) * 2.0
    o0 = torch.zeros(1, dtype=torch.int32, device=gpu)
    _, q0 = ops.conv2d_q(xq, am, codes, None, k, k, s, 0, wscale, shift, tile_cfg=base, emit_range=rng,
                         overflow=o0, want_f32=False)
    for c in pers:
        assert torch.equal(ops.conv2d_q(xq, am, codes, None, k, k, s, 0, wscale, shift, tile_cfg=c), ref), c
        o = torch.zeros(1, dtype=torch.int32, device=gpu)
        _, q = ops.conv2d_q(xq, am, codes, None, k, k, s, 0, wscale, shift, tile_cfg=c, emit_range=rng,
                            overflow=o, want_f32=False)
        assert torch.equal(q, q0) and torch.equal(o, o0), c


@pytest.mark.parametrize("shape", [(64, 64, 3, 1, 28, 16), (512, 128, 1, 1, 14, 64), (128, 80, 3, 2, 17, 24)],
                         ids=lambda s: "c%d_o%d_k%d_s%d_h%d_n%d" % s)
def test_persistent_general_epilogue_bitwise(gpu, shape):
    """The general epilogue (fp32 output, fp32 residual, per-image maxima by atomics, weight offsets)
    and 20 back-to-back launches of every persistent tile: the same bits every time."""
    from smpq import ops
    cin, cout, k, s, h, n = shape
    limbs = 3
    wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin * 3 + cout)
    g = torch.Generator().manual_seed(cout + n)
    x = torch.randn(n, h, h, cin, generator=g).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    ho = (h + 2 * (k // 2) - k) // s + 1
    res = torch.randn(n, ho, ho, cout, generator=g).to(gpu)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    base = _plain_cfgs(ops, limbs, 1, cout, cin, k)[0]
    ya0 = torch.zeros(n, device=gpu)
    y0 = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, residual=res, relu=True, y_absmax=ya0,
                      tile_cfg=base)
    pers = _persistent_cfgs(ops, limbs, 1, cout, cin, k)
    assert pers
    for c in pers:
        for _ in range(20):
            ya = torch.zeros(n, device=gpu)
            y = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, residual=res, relu=True,
                             y_absmax=ya, tile_cfg=c)
            assert torch.equal(y, y0) and torch.equal(ya, ya0), c
