"""GPU tests of the data-parallel contract (SURVEY.md 4 tier 4, 8(e)) and of the static-range
calibration bookkeeping: an image's logits do not depend on the batch or shard it runs in, and
two ranks whose calibration maxima are MAX-all-reduced produce, gathered, the single-GPU logits of
the global batch bit for bit (emulated in one process: the all-reduce is a torch.maximum)."""
import numpy as np
import pytest
import torch

from test_gpu import build_model

pytestmark = pytest.mark.gpu


def test_avgpool_fc_matches_torch_and_is_batch_invariant(gpu):
    from smpq import ops
    g = torch.Generator().manual_seed(3)
    feat = torch.relu(torch.randn(37, 7, 7, 2048, generator=g)).to(gpu)
    fc = torch.nn.Linear(2048, 1000).to(gpu)
    y = ops.avgpool_fc(feat, fc.weight, fc.bias)
    ref64 = feat.double().mean(dim=(1, 2)) @ fc.weight.double().T + fc.bias.double()
    assert (y.double() - ref64).abs().max().item() <= 1e-5 * ref64.abs().max().item()
    # the same bits whatever the batch around an image
    for s0, s1 in ((0, 1), (5, 21), (16, 37), (3, 4)):
        part = ops.avgpool_fc(feat[s0:s1].contiguous(), fc.weight, fc.bias)
        assert torch.equal(part, y[s0:s1])
    # no bias, odd sizes
    fc2 = torch.nn.Linear(64, 10, bias=False).to(gpu)
    f2 = torch.randn(3, 2, 3, 64, generator=g).to(gpu)
    y2 = ops.avgpool_fc(f2, fc2.weight, None)
    torch.testing.assert_close(y2, fc2(f2.mean(dim=(1, 2))), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode", ["static", "dynamic"])
@pytest.mark.parametrize("arch,assign", [("resnet50", "r50_mixed"), ("resnet18", "r18_u8")])
def test_sharded_logits_equal_single_gpu_bitwise(gpu, arch, assign, mode):
    """Two 'ranks' (shards of 5 and 5 images of a global batch of 10) vs the single-GPU forward of
    all 10: static mode with each shard's calibration maxima MAX-reduced (what engine.calibrate does
    under set_dp_group) — the reduced maxima equal the global batch's and the concatenated shard
    logits equal the global logits bit for bit; dynamic mode: per-image ranges, equal directly.
    Eager and graph-replayed, with the batch slices on concurrent streams."""
    from smpq import engine
    net = build_model(gpu, arch, assign)
    x = torch.randn(10, 3, 224, 224, generator=torch.Generator().manual_seed(41)).to(gpu)
    shards = [x[:5].contiguous(), x[5:].contiguous()]
    engine.set_range_mode(mode)
    old_graph = engine.USE_GRAPH[0]
    try:
        with torch.no_grad():
            for graph in (False, True):
                engine.USE_GRAPH[0] = graph
                if mode == "static":
                    cs = [engine.calibration_maxima(net, s) for s in shards]
                    assert cs[0].keys == cs[1].keys
                    red = torch.maximum(cs[0].maxima, cs[1].maxima)  # the MAX all-reduce of 2 ranks
                    cg = engine.calibration_maxima(net, x)
                    assert cg.keys == cs[0].keys and torch.equal(cg.maxima, red)
                    cs[0].maxima = red
                    engine.set_calibration(net, cs[0], widen=False)
                    parts = [net(s) for s in shards] + [net(s) for s in shards]  # eager/capture, replay
                    engine.set_calibration(net, cg, widen=False)
                    full = [net(x), net(x)]
                else:
                    parts = [net(s) for s in shards] * 2
                    full = [net(x)] * 2
                for k in range(2):
                    assert torch.equal(torch.cat(parts[2 * k:2 * k + 2]), full[k]), (graph, k)
    finally:
        engine.set_range_mode("static")
        engine.USE_GRAPH[0] = old_graph


def test_overflow_rerun_only_widens_ranges(gpu):
    """an overflow rerun keeps every static range at or above its previous value and
    does not invalidate the packed weights (no repack, no content-generation bump)."""
    from smpq import engine, stats
    net = build_model(gpu, "resnet18", "r18_u8")
    x = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(12)).to(gpu)
    with torch.no_grad():
        net(x)
        r0 = dict(net._smpq_ranges[0])
        rep0, o0 = stats["repack"], stats["overflow_reruns"]
        gens = [m._content_gen for m in net.modules() if hasattr(m, "_content_gen")]
        net(torch.cat([x[:3], 6 * x[3:]]))  # one image overflows the calibrated ranges
        assert stats["overflow_reruns"] == o0 + 1
        r1 = net._smpq_ranges[0]
        assert set(r1) == set(r0) and all(r1[k] >= r0[k] for k in r0)
        assert any(r1[k] > r0[k] for k in r0)
        net(0.5 * x)  # well inside: no further change
        assert net._smpq_ranges[0] == r1 and stats["overflow_reruns"] == o0 + 1
    assert stats["repack"] == rep0
    assert [m._content_gen for m in net.modules() if hasattr(m, "_content_gen")] == gens


def test_dynamic_forward_keeps_static_calibration(gpu):
    """a dynamic-range forward does not discard the static calibration (no
    recalibration and no repack when switching back), while a real content change still does."""
    import functions
    from smpq import engine, stats
    net = build_model(gpu, "resnet18", "r18_u8")
    x = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(13)).to(gpu)
    with torch.no_grad():
        net(x)
        a = net(x)
        c0, rep0 = stats["calibrations"], stats["repack"]
        engine.set_range_mode("dynamic")
        try:
            net(x)
        finally:
            engine.set_range_mode("static")
        b = net(x)
        assert stats["calibrations"] == c0 and stats["repack"] == rep0
        assert torch.equal(a, b)
        functions.channel_wise_quantizationperchan(net.layer2[0].conv1.weight.data, 4, 7)
        net(x)
        assert stats["calibrations"] == c0 + 1


def test_static_forward_refuses_caller_capture(gpu, monkeypatch):
    """inside a caller's graph capture the static forward cannot read its overflow /
    staleness flags, so it raises instead of returning possibly clamped or stale logits (the
    capture state is simulated: no real capture is left half-open by the exception)."""
    net = build_model(gpu, "resnet18", "r18_u8")
    x = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(14)).to(gpu)
    with torch.no_grad():
        net(x)
        monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
        with pytest.raises(RuntimeError, match="capture"):
            net(x)
        monkeypatch.undo()
        np.testing.assert_array_equal(net(x).shape, (2, 1000))

