"""Weight-stationary 1x1 tiles (csrc/conv_resident.hip, tile kind TILE_RESIDENT1X1): their
static-range limb-plane outputs and overflow flags equal the LDS-DMA kernel's bit for bit — 24-bit
fixed-point (3-limb) weights as in the downsample convs and exact codes (1 limb), with and without
ReLU, with a limb-plane residual, with weight offsets, stride 1 and 2, K 64 .. 1024, partial last
tiles, several tiles per workgroup, in range and overflowing —
and the calls they do not run are refused before launching. Every call goes through the C-ABI."""
import pytest
import torch

from test_gpu import make_layer

pytestmark = pytest.mark.gpu


def _res_cfgs(ops):
    return [c for c in ops.tile_configs() if ops.tile_kind(c) == ops.TILE_RESIDENT1X1]


def _layer(gpu, wl, seed, cin=64, cout=256):
    from smpq import ops
    if wl == 1:
        wd, step, codes, offset = make_layer(gpu, cin, cout, 1, seed=seed, bits_choice=(6, 4))
        return codes, None, step
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(cout, cin, 1, 1, generator=g) * 0.1).to(gpu)
    codes, offset, wscale, st = ops.pack_weights_ex(w, None, 3)
    return codes, None, wscale


@pytest.mark.parametrize("wl", [3, 1])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("cin,cout,n,h,stride", [
    (64, 256, 3, 56, 1), (64, 256, 2, 13, 1), (64, 256, 1, 5, 1), (64, 256, 2, 28, 2), (64, 256, 5, 9, 2),
    # the strided downsamples of layers 2 and 3 (K 256 / 512: several 64-B chunks per row), a
    # two-slab output (cout 128) and partial tiles
    (256, 512, 2, 56, 2), (512, 1024, 3, 28, 2), (256, 128, 3, 11, 1), (512, 64, 1, 7, 1),
    # the Bottleneck reductions (conv1: K 256 .. 1024) and a K-128 expansion without its residual
    (256, 64, 2, 21, 1), (1024, 256, 2, 14, 1), (128, 512, 1, 9, 1)])
def test_resident_equals_lds_dma(gpu, wl, relu, cin, cout, n, h, stride):
    from smpq import ops
    cfgs = [c for c in _res_cfgs(ops) if ops._tile_fits(c, 3, wl, cout, cin, 1)]
    assert len(_res_cfgs(ops)) == 4
    if not cfgs:  # K 1024 with 3 weight limbs: over the register budget (not a downsample shape)
        assert wl == 3 and cin == 1024
        return
    codes, offset, scale = _layer(gpu, wl, 7 * n + h + wl + cin, cin, cout)
    if wl == 3 and relu:  # built for the downsamples only: refused before launching
        from smpq import _lib
        xq = ops.act_quantize(torch.ones(n, h, h, cin, device=gpu), torch.ones(n, device=gpu), 3)
        with pytest.raises(_lib.SmpqError, match="resident"):
            ops.conv2d_q(xq, torch.ones(n, device=gpu), codes, offset, 1, 1, stride, 0, scale,
                         torch.zeros(cout, device=gpu), relu=True, tile_cfg=cfgs[0], emit_range=1.0,
                         overflow=torch.zeros(1, dtype=torch.int32, device=gpu), want_f32=False)
        return
    g = torch.Generator().manual_seed(h + 11 * n)
    x = torch.relu(torch.randn(n, h, h, cin, generator=g)).to(gpu)
    x[0] *= 3.0
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    shift = torch.linspace(-0.5, 0.5, cout, device=gpu)
    ref = ops.conv2d_q(xq, am, codes, offset, 1, 1, stride, 0, scale, shift, relu=relu)
    for frac in (2.0, 0.4):
        rng = float(ref.abs().max()) * frac
        ovf0 = torch.zeros(1, dtype=torch.int32, device=gpu)
        _, yq0 = ops.conv2d_q(xq, am, codes, offset, 1, 1, stride, 0, scale, shift, relu=relu, tile_cfg=-1,
                              emit_range=rng, overflow=ovf0, want_f32=False)
        assert int(ovf0.item()) == (1 if frac < 1 else 0)
        for c in cfgs:
            for _ in range(3):  # repeated launches: no race between a tile's DMA and the last one's reads
                ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
                _, yq = ops.conv2d_q(xq, am, codes, offset, 1, 1, stride, 0, scale, shift, relu=relu, tile_cfg=c,
                                     emit_range=rng, overflow=ovf, want_f32=False)
                assert torch.equal(yq, yq0), (c, frac)
                assert torch.equal(ovf, ovf0), (c, frac)


@pytest.mark.parametrize("cin,cout,n,h", [
    # the Bottleneck expansions conv3 + identity (resnet.py:111-113), partial last tiles
    (64, 256, 2, 56), (64, 256, 1, 5), (128, 512, 2, 28), (256, 1024, 3, 14), (512, 2048, 1, 7), (256, 128, 2, 9)])
def test_resident_residual_equals_lds_dma(gpu, cin, cout, n, h):
    """conv + BN + limb-plane residual + ReLU with exact-code weights: the residual tile arrives by
    LDS-DMA one tile ahead; limb planes and overflow flag bitwise the LDS-DMA kernel's, in range
    and overflowing, residual range above and below the output's."""
    from smpq import ops
    cfgs = [c for c in _res_cfgs(ops) if ops._tile_fits(c, 3, 1, cout, cin, 1)]
    assert cfgs
    codes, offset, scale = _layer(gpu, 1, 3 * n + h + cin, cin, cout)
    g = torch.Generator().manual_seed(h + 5 * n + cout)
    x = torch.relu(torch.randn(n, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    shift = torch.linspace(-0.5, 0.5, cout, device=gpu)
    r = torch.relu(torch.randn(n, h, h, cout, generator=g)).to(gpu)
    ref = ops.conv2d_q(xq, am, codes, offset, 1, 1, 1, 0, scale, shift, relu=True)
    for rr, frac in ((float(r.abs().max()) * 1.5, 2.0), (float(r.abs().max()) * 1.01, 0.5), (40.0, 2.0)):
        rq = ops.act_quantize(r, torch.full((n,), rr, device=gpu), 3)
        rng = (float(ref.abs().max()) + rr) * frac
        ovf0 = torch.zeros(1, dtype=torch.int32, device=gpu)
        _, yq0 = ops.conv2d_q(xq, am, codes, offset, 1, 1, 1, 0, scale, shift, relu=True, tile_cfg=-1,
                              emit_range=rng, overflow=ovf0, want_f32=False, residual_q=rq, residual_range=rr)
        for c in cfgs:
            for _ in range(2):
                ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
                _, yq = ops.conv2d_q(xq, am, codes, offset, 1, 1, 1, 0, scale, shift, relu=True, tile_cfg=c,
                                     emit_range=rng, overflow=ovf, want_f32=False, residual_q=rq,
                                     residual_range=rr)
                assert torch.equal(yq, yq0), (c, rr, frac)
                assert torch.equal(ovf, ovf0), (c, rr, frac)


@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("cin,cout,n,h", [(64, 256, 2, 28), (256, 64, 2, 21), (256, 1024, 1, 14), (1024, 256, 2, 7)])
def test_resident_weight_offsets_equal_lds_dma(gpu, cin, cout, n, h, res):
    """Exact codes off-centre (per-channel weight offsets, ReLU; with and without the residual):
    the v_dot4 digit-sum correction gives the LDS-DMA kernel's limb planes bit for bit."""
    from smpq import ops
    cfgs = [c for c in _res_cfgs(ops) if ops._tile_fits(c, 3, 1, cout, cin, 1)]
    assert cfgs
    codes, _, scale = _layer(gpu, 1, 11 * n + h + cin, cin, cout)
    g = torch.Generator().manual_seed(n + 13 * h)
    off = torch.randint(-100, 100, (cout,), generator=g, dtype=torch.int32).to(gpu)
    x = torch.relu(torch.randn(n, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    shift = torch.linspace(-0.5, 0.5, cout, device=gpu)
    kw = {}
    if res:
        r = torch.relu(torch.randn(n, h, h, cout, generator=g)).to(gpu)
        kw = dict(residual_q=ops.act_quantize(r, torch.full((n,), 5.0, device=gpu), 3), residual_range=5.0)
    ref = ops.conv2d_q(xq, am, codes, off, 1, 1, 1, 0, scale, shift, relu=True, **kw)
    for frac in (2.0, 0.4):
        rng = float(ref.abs().max()) * frac
        ovf0 = torch.zeros(1, dtype=torch.int32, device=gpu)
        _, yq0 = ops.conv2d_q(xq, am, codes, off, 1, 1, 1, 0, scale, shift, relu=True, tile_cfg=-1, emit_range=rng,
                              overflow=ovf0, want_f32=False, **kw)
        for c in cfgs:
            ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
            _, yq = ops.conv2d_q(xq, am, codes, off, 1, 1, 1, 0, scale, shift, relu=True, tile_cfg=c, emit_range=rng,
                                 overflow=ovf, want_f32=False, **kw)
            assert torch.equal(yq, yq0), (c, frac)
            assert torch.equal(ovf, ovf0), (c, frac)


def test_resident_many_tiles_per_workgroup(gpu):
    """More tiles than resident workgroups (each walks ~25 tiles), the R50 downsample's shape at a
    quarter of the batch: bitwise the LDS-DMA kernel's limb planes."""
    from smpq import ops
    codes, offset, scale = _layer(gpu, 3, seed=5)
    x = torch.relu(torch.randn(64, 56, 56, 64, generator=torch.Generator().manual_seed(9))).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    shift = torch.linspace(-0.1, 0.1, 256, device=gpu)
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    _, yq0 = ops.conv2d_q(xq, am, codes, offset, 1, 1, 1, 0, scale, shift, tile_cfg=-1, emit_range=8.0,
                          overflow=ovf, want_f32=False)
    for c in [c for c in _res_cfgs(ops) if ops._tile_fits(c, 3, 3, 256, 64, 1)]:
        _, yq = ops.conv2d_q(xq, am, codes, offset, 1, 1, 1, 0, scale, shift, tile_cfg=c, emit_range=8.0,
                             overflow=ovf, want_f32=False)
        assert torch.equal(yq, yq0), c
    assert int(ovf.item()) == 0


def test_resident_refuses_what_it_does_not_run(gpu):
    """fp32 outputs, a residual, weight offsets, pad > 0 and other shapes: SMPQ_E_INVALID before
    launching (the autotuner skips such calls); tile_supported reports the shape rule."""
    from smpq import _lib, ops
    c = _res_cfgs(ops)[0]
    assert ops._tile_fits(c, 3, 3, 256, 64, 1) and ops._tile_fits(c, 3, 1, 256, 64, 1)
    assert not ops._tile_fits(c, 3, 1, 128, 64, 1) and not ops._tile_fits(c, 3, 1, 256, 128, 1)
    assert not ops._tile_fits(c, 2, 1, 256, 64, 1) and not ops._tile_fits(c, 3, 1, 256, 64, 3)
    c2 = _res_cfgs(ops)[2]  # slab 64, K 128 .. 1024 (3 weight limbs: .. 512, the register budget)
    assert ops._tile_fits(c2, 3, 3, 512, 256, 1) and ops._tile_fits(c2, 3, 3, 1024, 512, 1)
    assert ops._tile_fits(c2, 3, 1, 256, 1024, 1) and not ops._tile_fits(c2, 3, 3, 256, 1024, 1)
    assert not ops._tile_fits(c2, 3, 1, 512, 2048, 1) and not ops._tile_fits(c2, 3, 3, 256, 192, 1)
    codes, offset, scale = _layer(gpu, 1, seed=3)
    x = torch.relu(torch.randn(1, 8, 8, 64, generator=torch.Generator().manual_seed(2))).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    shift = torch.zeros(256, device=gpu)
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    with pytest.raises(_lib.SmpqError, match="resident"):  # fp32 output
        ops.conv2d_q(xq, am, codes, offset, 1, 1, 1, 0, scale, shift, tile_cfg=c)
    rq = ops.act_quantize(torch.relu(torch.randn(1, 8, 8, 256, device=gpu)), torch.full((1,), 4.0, device=gpu), 3)
    with pytest.raises(_lib.SmpqError, match="resident"):  # limb-plane residual without ReLU
        ops.conv2d_q(xq, am, codes, offset, 1, 1, 1, 0, scale, shift, tile_cfg=c, emit_range=1.0, overflow=ovf,
                     want_f32=False, residual_q=rq, residual_range=4.0)
    with pytest.raises(_lib.SmpqError, match="resident"):  # an fp32 residual
        ops.conv2d_q(xq, am, codes, offset, 1, 1, 1, 0, scale, shift, tile_cfg=c, emit_range=1.0, overflow=ovf,
                     want_f32=False, relu=True, residual=torch.zeros(1, 8, 8, 256, device=gpu))
    with pytest.raises(_lib.SmpqError, match="resident"):  # pad 1
        ops.conv2d_q(xq, am, codes, offset, 1, 1, 1, 1, scale, shift, tile_cfg=c, emit_range=1.0, overflow=ovf,
                     want_f32=False)
    off = torch.zeros(256, dtype=torch.int32, device=gpu)
    off[3] = 5
    with pytest.raises(_lib.SmpqError, match="resident"):  # weight offsets without ReLU
        ops.conv2d_q(xq, am, codes, off, 1, 1, 1, 0, scale, shift, tile_cfg=c, emit_range=1.0, overflow=ovf,
                     want_f32=False)
