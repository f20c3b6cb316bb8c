"""`.pth` + bit-assignment sidecar (smpq/checkpoint.py): a state dict
written the reference's way (resnet50_main.py:212, fp32 weights only, no qbits/qstep) reloads with
its per-channel (bit, step) metadata recovered bitwise. CPU only: host quantizer in libsmpq.so."""
import numpy as np
import pytest
import torch


def _mixed_net(built_lib):
    import resnet
    from smpq.quant import quantize_layer_
    from smpq.assignments import addressable_convs
    torch.manual_seed(0)
    net = resnet.resnet18()
    rng = np.random.default_rng(1)
    for conv in addressable_convs(net)[:6]:
        bits = rng.choice([0, 2, 4, 6, 8], size=conv.out_channels)
        quantize_layer_(conv, bits)
    return net


def _plain(sd):
    return {k: v for k, v in sd.items() if not (k.endswith(".qbits") or k.endswith(".qstep"))}


def test_reference_pth_metadata_recovered(built_lib, tmp_path):
    import resnet
    from smpq import checkpoint
    net = _mixed_net(built_lib)
    p = tmp_path / "ref.pth"
    torch.save(_plain(net.state_dict()), p)  # what the reference's drivers write
    net2 = resnet.resnet18()
    got = checkpoint.load_checkpoint(net2, p, strict=False)
    want = checkpoint.bit_assignment(net)
    for ln in want:
        # recovered bits never exceed the recorded ones (a coarser grid may coincide exactly),
        # and every recorded channel is recovered
        w, g = np.asarray(want[ln]), np.asarray(got[ln])
        assert ((g > 0) == (w > 0)).all(), ln
        assert (g <= w).all(), ln
    sd1, sd2 = net.state_dict(), net2.state_dict()
    for k in sd1:
        if k.endswith(".weight"):
            assert torch.equal(sd1[k], sd2[k]), k


def test_sidecar_roundtrip_restores_bits_and_steps(built_lib, tmp_path):
    import resnet
    from smpq import checkpoint
    from smpq.assignments import addressable_convs
    net = _mixed_net(built_lib)
    p = tmp_path / "smpq.pth"
    checkpoint.save_checkpoint(net, p)
    side = checkpoint.read_sidecar(p)
    assert sorted(side) == list(range(1, 17))
    # strip the metadata from the .pth: the sidecar alone must restore it bitwise
    torch.save(_plain(torch.load(p, weights_only=True)), p)
    net2 = resnet.resnet18()
    got = checkpoint.load_checkpoint(net2, p, strict=False)
    assert got == checkpoint.bit_assignment(net)
    for a, b in zip(addressable_convs(net), addressable_convs(net2)):
        assert torch.equal(a.qbits, b.qbits)
        assert torch.equal(a.qstep, b.qstep)


def test_native_pth_keeps_metadata(built_lib, tmp_path):
    import resnet
    from smpq import checkpoint
    from smpq.assignments import addressable_convs
    net = _mixed_net(built_lib)
    p = tmp_path / "n.pth"
    checkpoint.save_checkpoint(net, p)
    net2 = resnet.resnet18()
    checkpoint.load_checkpoint(net2, p)
    for a, b in zip(addressable_convs(net), addressable_convs(net2)):
        assert torch.equal(a.qbits, b.qbits) and torch.equal(a.qstep, b.qstep)


@pytest.mark.gpu
def test_reference_pth_runs_exact_int8_path(gpu, tmp_path):
    """A reference-written .pth of the published R50 assignment (resnet50_main.py:426-427) loads
    back onto the exact int8 path of every addressable conv, with the same logits."""
    import resnet
    from smpq import assignments, checkpoint, engine
    torch.manual_seed(0)
    net = resnet.resnet50().to(gpu).eval()
    assignments.apply_assignment(net, "r50_mixed", semantics="cpu")
    p = tmp_path / "r50.pth"
    torch.save(_plain(net.state_dict()), p)
    torch.manual_seed(1)
    net2 = resnet.resnet50().to(gpu).eval()
    checkpoint.load_checkpoint(net2, p, map_location=gpu, strict=False)
    convs = assignments.addressable_convs(net2)
    kinds = [c.packed()[4] for c in convs]
    assert kinds == [c.packed()[4] for c in assignments.addressable_convs(net)]
    assert "exact8" in kinds
    x = torch.randn(8, 3, 224, 224, generator=torch.Generator().manual_seed(3)).to(gpu)
    engine.set_range_mode("dynamic")
    try:
        with torch.no_grad():
            a, b = net(x), net2(x)
    finally:
        engine.set_range_mode("static")
    # the weights are reproduced bitwise; a recovered step may differ from the recorded one by an
    # ulp (both reproduce every weight), which only moves the fp32 epilogue scale: the model-level
    # bound of test_gpu.LOGIT_RTOL[3] (2e-4 of max |logit|), and identical top-1
    assert (a - b).abs().max().item() <= 2e-4 * a.abs().max().item()
    assert torch.equal(a.argmax(1), b.argmax(1))


def test_sidecar_shape_mismatch_is_loud(built_lib, tmp_path):
    import json
    import resnet
    from smpq import checkpoint
    net = _mixed_net(built_lib)
    p = tmp_path / "bad.pth"
    checkpoint.save_checkpoint(net, p)
    torch.save(_plain(torch.load(p, weights_only=True)), p)
    side = json.load(open(checkpoint.sidecar_path(p)))
    side["convs"]["1"] = side["convs"]["1"][:-1]
    json.dump(side, open(checkpoint.sidecar_path(p), "w"))
    with pytest.raises(ValueError):
        checkpoint.load_checkpoint(resnet.resnet18(), p, strict=False)


def test_plain_pth_has_reference_keys_only(built_lib, tmp_path):
    # save_checkpoint's default .pth is the reference's format: no qbits/qstep keys, so the
    # reference's / torchvision's load_state_dict(strict=True) accepts it; strict loading here too
    import resnet
    from smpq import checkpoint
    net = _mixed_net(built_lib)
    p = tmp_path / "plain.pth"
    checkpoint.save_checkpoint(net, p)
    sd = torch.load(p, weights_only=True)
    assert not any(k.endswith((".qbits", ".qstep")) for k in sd)
    assert set(sd) == set(_plain(net.state_dict()))
    net2 = resnet.resnet18()
    checkpoint.load_checkpoint(net2, p, strict=True)
    # a key the model does not have is still an error under strict=True
    sd["bogus.weight"] = torch.zeros(1)
    torch.save(sd, p)
    with pytest.raises(RuntimeError):
        checkpoint.load_checkpoint(resnet.resnet18(), p, strict=True)


def test_sidecar_v2_restores_steps_bitwise(built_lib, tmp_path):
    import resnet
    from smpq import checkpoint
    from smpq.assignments import addressable_convs
    net = _mixed_net(built_lib)
    p = tmp_path / "v2.pth"
    checkpoint.save_checkpoint(net, p)
    steps = checkpoint.read_sidecar_steps(p)
    for ln, conv in enumerate(addressable_convs(net), start=1):
        assert np.array_equal(steps[ln].view(np.uint32), conv.qstep.numpy().view(np.uint32)), ln
    net2 = resnet.resnet18()
    checkpoint.load_checkpoint(net2, p)
    for a, b in zip(addressable_convs(net), addressable_convs(net2)):
        assert torch.equal(a.qbits, b.qbits)
        assert torch.equal(a.qstep.view(torch.int32), b.qstep.view(torch.int32))
        assert (a._bits_host == b._bits_host).all()


@pytest.mark.gpu
def test_sidecar_v2_logits_bitwise(gpu, tmp_path):
    """With the exact steps from the sidecar, a reloaded R50 mixed model's logits equal the
    original's bit for bit (no ulp-shifted recovered steps)."""
    import resnet
    from smpq import assignments, checkpoint, engine
    torch.manual_seed(0)
    net = resnet.resnet50().to(gpu).eval()
    assignments.apply_assignment(net, "r50_mixed", semantics="cpu")
    p = tmp_path / "r50v2.pth"
    checkpoint.save_checkpoint(net, p)
    torch.manual_seed(1)
    net2 = resnet.resnet50().to(gpu).eval()
    checkpoint.load_checkpoint(net2, p, map_location=gpu)
    x = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(3)).to(gpu)
    engine.set_range_mode("dynamic")
    try:
        with torch.no_grad():
            a, b = net(x), net2(x)
    finally:
        engine.set_range_mode("static")
    assert torch.equal(a, b)
