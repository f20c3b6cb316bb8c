"""The chained Bottleneck tails (csrc/conv_resident.hip, smpq_conv2d_pair_fwd / _chain_fwd): a
block's conv3 (+ identity, ReLU) and the next block's conv1 (ReLU) in one launch, and conv3 with
its 1x1 downsample computed in the same tiles (its output never written), give every output's limb
planes and the overflow flag bit for bit as the separate launches — in range and with any output
overflowing (the downsample's included), conv3 weight offsets, partial last tiles, many tiles per
workgroup — and the R50 forward with the chains on equals the forward without them (eager and
graph-replayed). Every call goes through the C-ABI."""
import pytest
import torch

from test_gpu import build_model, make_layer

pytestmark = pytest.mark.gpu


def _chain(gpu, cin, cout1, cout2, n, h, seed):
    from smpq import ops
    _, _, codes1, _ = make_layer(gpu, cin, cout1, 1, seed=seed, bits_choice=(8, 6, 4))
    _, _, codes2, _ = make_layer(gpu, cout1, cout2, 1, seed=seed + 1, bits_choice=(6, 4))
    g = torch.Generator().manual_seed(seed + 2)
    x = torch.relu(torch.randn(n, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    r = torch.relu(torch.randn(n, h, h, cout1, generator=g)).to(gpu)
    rr = float(r.abs().max()) * 1.25
    rq = ops.act_quantize(r, torch.full((n,), rr, device=gpu), 3)
    cs1 = (torch.rand(cout1, generator=g) * 0.02 + 0.01).to(gpu)
    sh1 = torch.linspace(-0.3, 0.3, cout1).to(gpu)
    cs2 = (torch.rand(cout2, generator=g) * 0.02 + 0.01).to(gpu)
    sh2 = torch.linspace(-0.2, 0.4, cout2).to(gpu)
    return xq, am, codes1, cs1, sh1, rq, rr, codes2, cs2, sh2


def _decode(yq):
    """The int24 codes of [3, ...] balanced limb planes."""
    return yq[0].long() + 256 * yq[1].long() + 65536 * yq[2].long()


def _two_launches(ops, gpu, xq, am, codes1, cs1, sh1, rq, rr, rng1, codes2, cs2, sh2, rng2):
    n = xq.shape[1]
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    _, y1 = ops.conv2d_q(xq, am, codes1, None, 1, 1, 1, 0, cs1, sh1, relu=True, emit_range=rng1, overflow=ovf,
                         want_f32=False, residual_q=rq, residual_range=rr)
    am1 = torch.full((n,), rng1, device=gpu)
    _, y2 = ops.conv2d_q(y1, am1, codes2, None, 1, 1, 1, 0, cs2, sh2, relu=True, emit_range=rng2, overflow=ovf,
                         want_f32=False)
    return y1, y2, ovf, am1


@pytest.mark.parametrize("cin,cout1,cout2,n,h", [
    (64, 256, 64, 2, 56), (64, 256, 64, 3, 9), (64, 256, 64, 1, 3), (64, 256, 64, 5, 14),
    # layer 1's last conv3 with layer 2's first conv1
    (64, 256, 128, 2, 56), (64, 256, 128, 3, 9)])
def test_pair_equals_two_launches(gpu, cin, cout1, cout2, n, h):
    from smpq import ops
    assert ops.conv_pair_supported(cin, cout1, cout2)
    xq, am, codes1, cs1, sh1, rq, rr, codes2, cs2, sh2 = _chain(gpu, cin, cout1, cout2, n, h, 3 * h + n)
    # the outputs' magnitudes, from a run with wide ranges
    y1w, y2w, ovw, _ = _two_launches(ops, gpu, xq, am, codes1, cs1, sh1, rq, rr, 1e4, codes2, cs2, sh2, 1e4)
    assert int(ovw.item()) == 0
    m1 = float(_decode(y1w).abs().max()) * 1e4 / 8323072 + 1e-3
    m2 = float(_decode(y2w).abs().max()) * 1e4 / 8323072 + 1e-3
    for f1, f2 in ((2.0, 2.0), (0.5, 2.0), (2.0, 0.5), (1.2, 1.1)):
        rng1, rng2 = m1 * f1, m2 * f2
        y1, y2, ovf0, am1 = _two_launches(ops, gpu, xq, am, codes1, cs1, sh1, rq, rr, rng1, codes2, cs2, sh2, rng2)
        if f1 < 1 or f2 < 1:
            assert int(ovf0.item()) == 1
        for _ in range(3):  # repeated launches: no race between tiles
            ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
            p1, p2 = ops.conv_pair_q(xq, am, codes1, cs1, sh1, rq, rr, rng1, am1, codes2, cs2, sh2, rng2, ovf)
            assert torch.equal(p1, y1), (f1, f2)
            assert torch.equal(p2, y2), (f1, f2)
            assert torch.equal(ovf, ovf0), (f1, f2)


def _ds_case(gpu, n, h, seed, offsets, cin=64, cout=256, ds_cin=64, hd=None):
    """The first block of a stage: x (ds_cin ch, hd x hd) -> downsample ds_cin -> cout (24-bit
    fixed-point weights, no ReLU, stride hd / h) and t2 (cin ch, h x h) -> conv3 cin -> cout (+ the
    downsample's output, ReLU) [-> next conv1 cout -> 64]."""
    from smpq import ops
    hd = hd or h
    xq, am, codes1, cs1, sh1, rq, rr, codes2, cs2, sh2 = _chain(gpu, cin, cout, 64, n, h, seed)
    g = torch.Generator().manual_seed(seed + 7)
    xb = torch.relu(torch.randn(n, hd, hd, ds_cin, generator=g)).to(gpu)
    amb = ops.act_absmax(xb)
    xbq = ops.act_quantize(xb, amb, 3)
    wds = (torch.randn(cout, ds_cin, 1, 1, generator=g) * 0.1).to(gpu)
    dcodes, _, dscale, _ = ops.pack_weights_ex(wds, None, 3)
    dcs = (dscale * (torch.rand(cout, generator=g) + 0.5).to(gpu)).contiguous()
    dsh = torch.linspace(-0.2, 0.2, cout).to(gpu)
    off = None
    if offsets:
        off = torch.randint(-90, 90, (cout,), generator=g, dtype=torch.int32).to(gpu)
    return xq, am, codes1, off, cs1, sh1, codes2, cs2, sh2, xbq, amb, dcodes, dcs, dsh


def _separate(ops, gpu, xq, am, codes1, off, cs1, sh1, codes2, cs2, sh2, xbq, amb, dcodes, dcs, dsh,
              rng_d, rng1, rng2, with_next, st=1):
    n = xq.shape[1]
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    _, yd = ops.conv2d_q(xbq, amb, dcodes, None, 1, 1, st, 0, dcs, dsh, relu=False, emit_range=rng_d, overflow=ovf,
                         want_f32=False)
    _, y1 = ops.conv2d_q(xq, am, codes1, off, 1, 1, 1, 0, cs1, sh1, relu=True, emit_range=rng1, overflow=ovf,
                         want_f32=False, residual_q=yd, residual_range=rng_d)
    am1 = torch.full((n,), rng1, device=gpu)
    y2 = None
    if with_next:
        _, y2 = ops.conv2d_q(y1, am1, codes2, None, 1, 1, 1, 0, cs2, sh2, relu=True, emit_range=rng2, overflow=ovf,
                             want_f32=False)
    return y1, y2, ovf, am1


@pytest.mark.parametrize("offsets", [False, True])
@pytest.mark.parametrize("cin,cout,ds_cin,st,n,h,hd", [
    (64, 256, 64, 1, 2, 56, 56), (64, 256, 64, 1, 3, 9, 9), (64, 256, 64, 1, 1, 3, 3), (64, 256, 64, 1, 16, 28, 28),
    # layer2 / layer3 block 0: the strided downsample (even and odd input sizes), partial tiles
    (128, 512, 256, 2, 2, 28, 56), (128, 512, 256, 2, 3, 5, 9), (256, 1024, 512, 2, 2, 14, 28),
    (256, 1024, 512, 2, 1, 3, 5)])
def test_chain_fused_downsample_equals_separate_launches(gpu, cin, cout, ds_cin, st, n, h, hd, offsets):
    with_next = False  # (built without the chained conv1: refused below)
    from smpq import ops
    assert ops.conv_chain_supported(64, 256, 64) and ops.conv_chain_ds_supported(cin, cout, ds_cin, st)
    xq, am, codes1, off, cs1, sh1, codes2, cs2, sh2, xbq, amb, dcodes, dcs, dsh = _ds_case(
        gpu, n, h, 5 * h + n, offsets, cin, cout, ds_cin, hd)
    w = _separate(ops, gpu, xq, am, codes1, off, cs1, sh1, codes2, cs2, sh2, xbq, amb, dcodes, dcs, dsh,
                  1e4, 1e4, 1e4, True, st)
    assert int(w[2].item()) == 0
    # the magnitudes of the three outputs (wide-range run), then ranges around them
    _, ydw = ops.conv2d_q(xbq, amb, dcodes, None, 1, 1, st, 0, dcs, dsh, emit_range=1e4,
                          overflow=torch.zeros(1, dtype=torch.int32, device=gpu), want_f32=False)
    md = float(_decode(ydw).abs().max()) * 1e4 / 8323072 + 1e-3
    m1 = float(_decode(w[0]).abs().max()) * 1e4 / 8323072 + 1e-3
    m2 = float(_decode(w[1]).abs().max()) * 1e4 / 8323072 + 1e-3
    for fd, f1, f2 in ((2.0, 2.0, 2.0), (0.5, 3.0, 3.0), (2.0, 0.5, 2.0), (2.0, 2.0, 0.5), (1.1, 1.3, 1.2)):
        rng_d, rng1, rng2 = md * fd, m1 * f1, m2 * f2
        y1, y2, ovf0, am1 = _separate(ops, gpu, xq, am, codes1, off, cs1, sh1, codes2, cs2, sh2, xbq, amb, dcodes,
                                      dcs, dsh, rng_d, rng1, rng2, with_next, st)
        if fd < 1 or f1 < 1 or (f2 < 1 and with_next):
            assert int(ovf0.item()) == 1, (fd, f1, f2)
        for _ in range(2):
            ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
            p1, p2 = ops.conv_chain_q(xq, am, codes1, off, cs1, sh1, rng1, am1, ovf,
                                      ds=(xbq, amb, dcodes, dcs, dsh, rng_d, st),
                                      nxt=(codes2, cs2, sh2, rng2) if with_next else None)
            assert torch.equal(p1, y1), (fd, f1, f2)
            assert (p2 is None) == (not with_next) and (p2 is None or torch.equal(p2, y2)), (fd, f1, f2)
            assert torch.equal(ovf, ovf0), (fd, f1, f2)
    if cin == 64:  # (with a chained conv1 too: not built)
        with pytest.raises(ValueError, match="shape not built"):
            ops.conv_chain_q(xq, am, codes1, off, cs1, sh1, 1.0, am, torch.zeros(1, dtype=torch.int32, device=gpu),
                             ds=(xbq, amb, dcodes, dcs, dsh, 1.0), nxt=(codes2, cs2, sh2, 1.0))


@pytest.mark.parametrize("with_next", [True, False])
def test_chain_offsets_with_limb_plane_identity(gpu, with_next):
    """conv3 with weight offsets and its identity as limb planes (the pair path)."""
    from smpq import ops
    xq, am, codes1, cs1, sh1, rq, rr, codes2, cs2, sh2 = _chain(gpu, 64, 256, 64, 2, 28, 17)
    off = torch.randint(-60, 60, (256,), generator=torch.Generator().manual_seed(3), dtype=torch.int32).to(gpu)
    ovf0 = torch.zeros(1, dtype=torch.int32, device=gpu)
    _, y1 = ops.conv2d_q(xq, am, codes1, off, 1, 1, 1, 0, cs1, sh1, relu=True, emit_range=50.0, overflow=ovf0,
                         want_f32=False, residual_q=rq, residual_range=rr)
    am1 = torch.full((2,), 50.0, device=gpu)
    _, y2 = ops.conv2d_q(y1, am1, codes2, None, 1, 1, 1, 0, cs2, sh2, relu=True, emit_range=50.0, overflow=ovf0,
                         want_f32=False)
    if not with_next:
        with pytest.raises(_lib_error()):  # nothing to chain: the plain conv3 is smpq_conv2d_fwd_q's
            ops.conv_chain_q(xq, am, codes1, off, cs1, sh1, 50.0, am1, ovf0, residual_q=rq, residual_range=rr)
        return
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    p1, p2 = ops.conv_chain_q(xq, am, codes1, off, cs1, sh1, 50.0, am1, ovf, residual_q=rq, residual_range=rr,
                              nxt=(codes2, cs2, sh2, 50.0))
    assert torch.equal(p1, y1) and torch.equal(p2, y2) and torch.equal(ovf, ovf0)


def _lib_error():
    from smpq import _lib
    return _lib.SmpqError


def test_pair_many_tiles(gpu):
    """The R50 layer1 shape at 64 images: every workgroup walks ~75 tiles."""
    from smpq import ops
    xq, am, codes1, cs1, sh1, rq, rr, codes2, cs2, sh2 = _chain(gpu, 64, 256, 64, 64, 56, 11)
    y1, y2, ovf0, am1 = _two_launches(ops, gpu, xq, am, codes1, cs1, sh1, rq, rr, 40.0, codes2, cs2, sh2, 40.0)
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    p1, p2 = ops.conv_pair_q(xq, am, codes1, cs1, sh1, rq, rr, 40.0, am1, codes2, cs2, sh2, 40.0, ovf)
    assert torch.equal(p1, y1) and torch.equal(p2, y2) and torch.equal(ovf, ovf0)


def test_pair_refuses_what_it_does_not_run(gpu):
    from smpq import _lib, ops
    assert not ops.conv_pair_supported(256, 1024, 256) and not ops.conv_pair_supported(64, 256, 192)
    assert not ops.conv_pair_supported(128, 512, 128)
    assert not ops.conv_pair_supported(64, 256, 64, 2)
    xq, am, codes1, cs1, sh1, rq, rr, codes2, cs2, sh2 = _chain(gpu, 64, 256, 64, 1, 4, 5)
    lib = _lib.load()
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    y1 = torch.empty(3, 1, 4, 4, 256, dtype=torch.int8, device=gpu)
    y2 = torch.empty(3, 1, 4, 4, 64, dtype=torch.int8, device=gpu)
    # no residual: refused before launching
    rc = lib.smpq_conv2d_pair_fwd(_lib.ptr(xq), _lib.ptr(am), 1, 4, 4, 64, _lib.ptr(codes1), 256, _lib.ptr(cs1),
                                  _lib.ptr(sh1), None, 0.0, _lib.ptr(y1), 1.0, _lib.ptr(am), _lib.ptr(codes2), 64,
                                  _lib.ptr(cs2), _lib.ptr(sh2), _lib.ptr(y2), 1.0, _lib.ptr(ovf), _lib.stream_ptr())
    assert rc == _lib.SMPQ_E_INVALID
    with pytest.raises(ValueError, match="pair"):  # a shape that is not built
        ops.conv_pair_q(xq, am, codes1[:128].contiguous(), cs1[:128].contiguous(), sh1[:128].contiguous(),
                        rq[..., :128].contiguous(), rr, 1.0, am, codes2[:, :128].contiguous(), cs2, sh2, 1.0, ovf)


@pytest.mark.parametrize("graph", [False, True])
def test_r50_forward_with_chains_bitwise(gpu, graph):
    """R50 mixed, static ranges, 2 batch slices: the forward with every chain on (layer1 block 0's
    fused downsample, the next-conv1 chains of blocks 1 and 2) gives the logits of the forward
    with none, bit for bit."""
    from smpq import engine, stats
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(37)).to(gpu)
    old = engine.PAIR_1X1[0], engine.FUSE_DS[0], engine.USE_GRAPH[0]
    try:
        with torch.no_grad():
            engine.USE_GRAPH[0] = False
            engine.PAIR_1X1[0] = engine.FUSE_DS[0] = False
            net(x)  # calibrate
            want = net(x)
            engine.PAIR_1X1[0] = engine.FUSE_DS[0] = True
            engine.USE_GRAPH[0] = graph
            f0, c0 = stats.get("fused_ds", 0), stats.get("chain_conv", 0)
            got = [net(x) for _ in range(3)]
            if not graph:
                # 3 forwards x 2 slices x the first blocks of layers 1-3 whose conv3 is exact codes
                # (+ the pairs of layer1 blocks 1 and 2 among the chains)
                fd, ch = stats.get("fused_ds", 0) - f0, stats.get("chain_conv", 0) - c0
                assert fd % 6 == 0 and fd >= 6 and ch == fd + 12, (fd, ch)  # + layer1 b1->b2, b2->layer2
            assert net.layer1[0].downsample[0].last_path.endswith("-chain")
            assert net.layer1[0].conv3.last_path.endswith("-chain")
    finally:
        engine.PAIR_1X1[0], engine.FUSE_DS[0], engine.USE_GRAPH[0] = old
    for g in got:
        assert torch.equal(g, want)


@pytest.mark.parametrize("graph", [False, True])
def test_r50_forward_with_pairs_bitwise(gpu, graph):
    """R50 mixed, static ranges, 2 batch slices: the forward with the pair launches (the two
    layer1 chains) gives the logits of the forward without them, bit for bit."""
    from smpq import engine, stats
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(31)).to(gpu)
    old = engine.PAIR_1X1[0], engine.USE_GRAPH[0], engine.FUSE_DS[0]
    try:
        with torch.no_grad():
            engine.USE_GRAPH[0] = False
            engine.FUSE_DS[0] = False  # (pairs only)
            engine.PAIR_1X1[0] = False
            net(x)  # calibrate
            want = net(x)
            engine.PAIR_1X1[0] = True
            engine.USE_GRAPH[0] = graph
            p0 = stats.get("pair_conv", 0)
            got = [net(x) for _ in range(3)]
            if not graph:
                # 3 forwards x 2 slices x the layer1 chains whose two convs are exact codes (in
                # r50_mixed one layer1 conv keeps unquantized channels: fixed point, unpaired)
                d = stats.get("pair_conv", 0) - p0
                assert d >= 6 and d % 6 == 0, d
            assert net.layer1[1].conv3.last_path.endswith("-chain")
    finally:
        engine.PAIR_1X1[0], engine.USE_GRAPH[0], engine.FUSE_DS[0] = old
    for g in got:
        assert torch.equal(g, want)
