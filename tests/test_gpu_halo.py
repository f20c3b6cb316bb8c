"""Halo-patch 3x3 kernel (csrc/conv_halo.hip, tile kind TILE_HALO3X3): its static-range limb-plane
outputs and overflow flags equal the implicit-GEMM kernel's bit for bit on every configuration,
for full and partial tiles, several input-channel chunks, 2 and 3 activation limbs, weight offsets,
both weight layouts, ReLU on and off, in range and overflowing. Every call goes through the C-ABI."""
import pytest
import torch

from test_gpu import make_layer

pytestmark = pytest.mark.gpu


def _halo_cfgs(ops, limbs, cin, cout):
    return [c for c in ops.tile_configs()
            if ops.tile_kind(c) == ops.TILE_HALO3X3 and ops._tile_fits(c, limbs, 1, cout, cin, 3)]


@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("limbs", [2, 3])
@pytest.mark.parametrize("shape", [(64, 64, 56, 56, 2), (128, 128, 28, 28, 3), (256, 256, 14, 14, 2),
                                   (64, 128, 13, 17, 2), (192, 64, 9, 30, 1), (64, 64, 13, 17, 3),
                                   # narrow images: 7 x 7 (an odd image count), width 16, narrower
                                   # than 7, a partial row tile
                                   (512, 512, 7, 7, 3), (64, 128, 9, 16, 2), (128, 64, 5, 6, 3)],
                         ids=lambda s: "c%d_o%d_%dx%d_n%d" % s)
def test_halo_equals_implicit_gemm(gpu, shape, limbs, relu):
    from smpq import _lib, ops
    cin, cout, h, w, n = shape
    wd, step, codes, offset = make_layer(gpu, cin, cout, 3, seed=cin + 3 * cout + h)
    g = torch.Generator().manual_seed(h * w)
    x = torch.relu(torch.randn(n, h, w, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    ref = ops.conv2d_q(xq, am, codes, offset, 3, 3, 1, 1, step, shift, relu=relu)
    cfgs = _halo_cfgs(ops, limbs, cin, cout)
    assert cfgs
    for frac in (2.0, 0.5):
        rng = float(ref.abs().max()) * frac
        for layout in ("auto", "rowmajor"):
            ovf0 = torch.zeros(1, dtype=torch.int32, device=gpu)
            _, yq0 = ops.conv2d_q(xq, am, codes, offset, 3, 3, 1, 1, step, shift, relu=relu, tile_cfg=-1,
                                  emit_range=rng, overflow=ovf0, want_f32=False, weight_layout=layout)
            assert int(ovf0.item()) == (1 if frac < 1 else 0)
            for c in cfgs:
                ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
                if not relu:  # the halo kernel runs the ReLU convs only (the autotuner skips it here)
                    with pytest.raises(_lib.SmpqError, match="halo"):
                        ops.conv2d_q(xq, am, codes, offset, 3, 3, 1, 1, step, shift, relu=relu, tile_cfg=c,
                                     emit_range=rng, overflow=ovf, want_f32=False, weight_layout=layout)
                    continue
                _, yq = ops.conv2d_q(xq, am, codes, offset, 3, 3, 1, 1, step, shift, relu=relu, tile_cfg=c,
                                     emit_range=rng, overflow=ovf, want_f32=False, weight_layout=layout)
                assert torch.equal(yq, yq0), (c, frac, layout)
                assert torch.equal(ovf, ovf0), (c, frac, layout)


@pytest.mark.parametrize("with_offset", [True, False])
@pytest.mark.parametrize("limbs", [2, 3])
@pytest.mark.parametrize("shape", [(64, 64, 56, 56, 2), (128, 128, 28, 28, 3), (256, 256, 14, 14, 2),
                                   (512, 512, 7, 7, 3), (64, 128, 13, 17, 2)],
                         ids=lambda s: "c%d_o%d_%dx%d_n%d" % s)
def test_halo_residual_equals_implicit_gemm(gpu, shape, limbs, with_offset):
    """BasicBlock conv2 (+ the identity as limb planes, then ReLU) on the halo tiles: the limb-plane
    outputs and overflow flags equal the implicit-GEMM kernel's bit for bit, in range and
    overflowing, with and without weight offsets."""
    from smpq import ops
    cin, cout, h, w, n = shape
    wd, step, codes, offset = make_layer(gpu, cin, cout, 3, seed=cin + cout + w)
    offset = offset if with_offset else None
    g = torch.Generator().manual_seed(h + 7 * w)
    x = torch.relu(torch.randn(n, h, w, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    r = torch.relu(torch.randn(n, h, w, cout, generator=g)).to(gpu)
    rrange = float(r.abs().max()) * 1.5
    rq = ops.act_quantize(r, torch.full((n,), rrange, device=gpu), limbs)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    kw = dict(relu=True, want_f32=False, residual_q=rq, residual_range=rrange)
    ref = ops.conv2d_q(xq, am, codes, offset, 3, 3, 1, 1, step, shift, relu=True)
    cfgs = _halo_cfgs(ops, limbs, cin, cout)
    assert cfgs
    for frac in (3.0, 0.5):
        rng = (float(ref.abs().max()) + rrange) * frac
        ovf0 = torch.zeros(1, dtype=torch.int32, device=gpu)
        _, yq0 = ops.conv2d_q(xq, am, codes, offset, 3, 3, 1, 1, step, shift, tile_cfg=-1, emit_range=rng,
                              overflow=ovf0, **kw)
        if frac < 1:
            assert int(ovf0.item()) == 1
        for c in cfgs:
            ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
            _, yq = ops.conv2d_q(xq, am, codes, offset, 3, 3, 1, 1, step, shift, tile_cfg=c, emit_range=rng,
                                 overflow=ovf, **kw)
            assert torch.equal(yq, yq0), (c, frac)
            assert torch.equal(ovf, ovf0), (c, frac)


def test_halo_without_offsets_and_repeatable(gpu):
    """No weight offsets (the plain-code path) and 20 back-to-back launches of every halo config
    give the same bits (no race between the DMA of one chunk and the reads of the last)."""
    from smpq import _lib, ops
    cin, cout, h = 128, 64, 28
    wd, step, codes, offset = make_layer(gpu, cin, cout, 3, seed=11, bits_choice=(6, 4))
    x = torch.relu(torch.randn(4, h, h, cin, generator=torch.Generator().manual_seed(3))).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    shift = torch.zeros(cout, device=gpu)
    ref = ops.conv2d_q(xq, am, codes, None, 3, 3, 1, 1, step, shift, relu=True)
    rng = float(ref.abs().max()) * 2
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    _, yq0 = ops.conv2d_q(xq, am, codes, None, 3, 3, 1, 1, step, shift, relu=True, emit_range=rng, overflow=ovf,
                          want_f32=False)
    for c in _halo_cfgs(ops, 3, cin, cout):
        outs = [ops.conv2d_q(xq, am, codes, None, 3, 3, 1, 1, step, shift, relu=True, tile_cfg=c, emit_range=rng,
                             overflow=ovf, want_f32=False)[1] for _ in range(20)]
        for yq in outs:
            assert torch.equal(yq, yq0), c
    assert int(ovf.item()) == 0


def test_halo_refuses_what_it_does_not_run(gpu):
    """Stride 2, fp32 outputs and no-ReLU convs are refused with SMPQ_E_INVALID (the autotuner
    skips such configurations), never run."""
    from smpq import _lib, ops
    cin, cout = 64, 64
    wd, step, codes, offset = make_layer(gpu, cin, cout, 3, seed=5)
    x = torch.relu(torch.randn(1, 8, 8, cin, generator=torch.Generator().manual_seed(6))).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    shift = torch.zeros(cout, device=gpu)
    c = _halo_cfgs(ops, 3, cin, cout)[0]
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    with pytest.raises(_lib.SmpqError, match="halo"):
        ops.conv2d_q(xq, am, codes, offset, 3, 3, 2, 1, step, shift, tile_cfg=c, emit_range=1.0, overflow=ovf,
                     want_f32=False)
    with pytest.raises(_lib.SmpqError, match="halo"):
        ops.conv2d_q(xq, am, codes, offset, 3, 3, 1, 1, step, shift, tile_cfg=c)


@pytest.mark.parametrize("arch,assign", [("resnet18", "r18_u8"), ("resnet50", "r50_mixed")])
def test_model_forward_halo_tiles_bitwise(gpu, arch, assign):
    """A whole static-range forward with every 3x3 / stride-1 conv on a halo tile gives the same
    logits, bit for bit, as with every conv on the implicit-GEMM tiles (and the halo kernel did
    run: its configurations were chosen for those convs)."""
    from smpq import engine, ops
    from test_gpu import build_model
    net = build_model(gpu, arch, assign, None)
    x = torch.randn(5, 3, 224, 224, generator=torch.Generator().manual_seed(7)).to(gpu)
    orig = ops._choose_tile
    picked = []

    def choose(kind):
        def pick(key, run, cands, variant=None):
            halo = [c for c in cands if ops.tile_kind(c) == ops.TILE_HALO3X3]
            gemm = [c for c in cands if ops.tile_kind(c) != ops.TILE_HALO3X3]
            # a halo tile only where the call is one it runs (lean, ReLU): key = n|h|w|cin|cout|kh|kw|
            # stride|pad|limbs|wlimbs|res_f32|emit_q|want_f32|res_q
            lean = key[5] == 3 and key[7] == 1 and key[12] and not key[13] and not key[11]
            if kind == "halo" and halo and lean:
                c = halo[0]
                picked.append(c)
                return c
            return gemm[0] if gemm else None
        return pick

    outs = {}
    try:
        engine.USE_GRAPH[0] = False
        for kind in ("gemm", "halo"):
            ops._TUNED.clear()
            ops._choose_tile = choose(kind)
            engine.new_evaluation(net)
            with torch.no_grad():
                net(x)  # calibration (dynamic ranges: the general epilogue, never a halo tile)
                outs[kind] = net(x).clone()
    finally:
        ops._choose_tile = orig
        ops._TUNED.clear()
        engine.USE_GRAPH[0] = True
    assert picked, "no conv ran on a halo tile"
    assert torch.equal(outs["halo"], outs["gemm"])
