"""The fused conv3 + next conv1 launch (smpq_conv2d_fwd_q_next, round 3): a Bottleneck's last conv
(+ limb-plane residual, + ReLU) and the next block's 1x1 conv1 in one launch, the first conv's output
tile kept in LDS as the second's operand. Both outputs must be bitwise those of the two separate
launches (resnet.py:104-111 then 102-104 of the next block), overflow flag included, on every
fused tile, with partial pixel tiles and weight offsets on the first conv."""
import pytest
import torch

from test_gpu import build_model

pytestmark = pytest.mark.gpu


def _codes(gpu, cin, cout, seed, bits_choice):
    """Exact one-limb codes of a random 1x1 conv quantized per channel with the given bit widths
    (8-bit channels may carry offsets): (wscale, codes, offset | None)."""
    from smpq import ops
    for s in range(seed, seed + 20):
        g = torch.Generator().manual_seed(s)
        w = (torch.randn(cout, cin, 1, 1, generator=g) * 0.05).to(gpu)
        bits = torch.tensor(bits_choice)[torch.randint(0, len(bits_choice), (cout,), generator=g)].tolist()
        step = ops.quantize_channels_(w.reshape(cout, -1), bits)
        codes, offset, wscale, st = ops.pack_weights_ex(w, step, 1)
        if st.cpu().tolist()[:2] == [0, 0]:
            if offset is not None and not bool((offset != 0).any()):
                offset = None
            return wscale, codes, offset
    raise AssertionError("no exact one-limb codes")


@pytest.mark.parametrize("shape", [(64, 256, 64, 20), (64, 256, 128, 11), (128, 512, 128, 13), (128, 512, 256, 7)],
                         ids=lambda s: "c%d_o%d_n%d_h%d" % s)
def test_conv_next_bitwise(gpu, shape):
    from smpq import ops
    cmid, cout, ncout, h = shape
    limbs, n = 3, 3
    g = torch.Generator().manual_seed(cmid + cout + ncout)
    step3, codes3, off3 = _codes(gpu, cmid, cout, cout + 1, (8, 6, 4))  # 8-bit channels: offsets
    step1, codes1, off1 = _codes(gpu, cout, ncout, ncout + 2, (6, 4))
    assert off1 is None
    x = torch.relu(torch.randn(n, h, h, cmid, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, limbs)
    rq = ops.act_quantize(torch.randn(n, h, h, cout, generator=g).clamp(-4, 4).to(gpu),
                          torch.full((n,), 4.0, device=gpu), limbs)
    cs3 = (step3 * torch.linspace(0.5, 1.5, cout, device=gpu)).contiguous()
    sh3 = torch.linspace(-0.2, 0.3, cout, device=gpu)
    cs1 = (step1 * torch.linspace(1.5, 0.5, ncout, device=gpu)).contiguous()
    sh1 = torch.linspace(-0.1, 0.2, ncout, device=gpu)
    big = torch.zeros(1, dtype=torch.int32, device=gpu)
    y3 = ops.conv2d_q(xq, am, codes3, off3, 1, 1, 1, 0, cs3, sh3, relu=True, residual_q=rq, residual_range=4.0)
    rng3 = float(y3.abs().max()) * 2.0
    ram = torch.full((n,), rng3, device=gpu)
    for tight in (False, True):
        o_ref = torch.zeros(1, dtype=torch.int32, device=gpu)
        _, q3 = ops.conv2d_q(xq, am, codes3, off3, 1, 1, 1, 0, cs3, sh3, relu=True, residual_q=rq, residual_range=4.0,
                             emit_range=rng3, overflow=o_ref, want_f32=False)
        y1 = ops.conv2d_q(q3, ram, codes1, None, 1, 1, 1, 0, cs1, sh1, relu=True)
        rng1 = float(y1.abs().max()) * (0.5 if tight else 2.0)  # tight: values beyond the range (overflow)
        _, q1 = ops.conv2d_q(q3, ram, codes1, None, 1, 1, 1, 0, cs1, sh1, relu=True, emit_range=rng1, overflow=o_ref,
                             want_f32=False)
        assert int(o_ref.item()) == (1 if tight else 0)
        cfgs = ops.next_tile_configs(cmid, cout, 1, ncout)
        assert cfgs, shape
        for c in cfgs:
            o = torch.zeros(1, dtype=torch.int32, device=gpu)
            f3, f1 = ops.conv2d_q_next(xq, am, codes3, off3, 1, 1, 1, 0, cs3, sh3, rng3, o, codes1, ram, cs1, sh1, rng1,
                                       residual_q=rq, residual_range=4.0, tile_cfg=c)
            assert torch.equal(f3, q3), (c, tight)
            assert torch.equal(f1, q1), (c, tight)
            assert torch.equal(o, o_ref), (c, tight)
    del big


def test_model_fused_next_bitwise(gpu):
    """R50 (mixed 8/6/4, BN-recalibrated parity model) static forward: logits with the fused
    conv3 + conv1 launches equal those of the separate launches bit for bit, eager and graph."""
    from smpq import engine
    net = build_model(gpu, "resnet50", "r50_mixed", "r50_mixed_cal")
    x = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(21)).to(gpu)
    old = engine.FUSE_NEXT[0], engine.USE_GRAPH[0]
    out = {}
    try:
        for fuse in (False, True):
            for graph in (False, True):
                engine.FUSE_NEXT[0], engine.USE_GRAPH[0] = fuse, graph
                with torch.no_grad():
                    net(x)
                    out[(fuse, graph)] = net(x).clone()
                if fuse:
                    fused = [m for m in net.modules() if getattr(m, "last_path", "") == "hip-exact8-fused-next"]
                    print("fused conv launches:", len(fused))
                    assert len(fused) >= 2
    finally:
        engine.FUSE_NEXT[0], engine.USE_GRAPH[0] = old
    ref = out[(False, False)]
    for k, v in out.items():
        assert torch.equal(v, ref), k
