"""Product model construction and assignment fixtures (CPU only, no kernel launches)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN


def _g():
    return np.load(os.path.join(GOLDEN, "model_goldens.npz"), allow_pickle=False)


@pytest.mark.parametrize("case,arch", [("r18_fp32", "resnet18"), ("r34_4bit", "resnet34"), ("r50_mixed", "resnet50")])
def test_seeded_weights_identical_to_reference(case, arch):
    """Same module order + init (resnet.py:165-170) => bit-identical seeded weights."""
    import resnet
    g = _g()
    torch.manual_seed(0)
    net = getattr(resnet, arch)()
    sd = net.state_dict()
    n = 0
    for k in g.files:
        if k.startswith(case + "/wsum/"):
            w = sd[k[len(case + "/wsum/"):]].double()
            np.testing.assert_array_equal([w.sum().item(), w.abs().sum().item()], g[k])
            n += 1
    assert n >= 17


def test_state_dict_keys_are_torchvision_plus_metadata():
    import resnet
    net = resnet.resnet50()
    keys = set(net.state_dict())
    assert "layer1.0.conv1.weight" in keys and "fc.bias" in keys and "layer1.0.downsample.0.weight" in keys
    extra = {k for k in keys if k.endswith(".qbits") or k.endswith(".qstep")}
    assert len(extra) == 2 * (48 + 4 + 1)  # addressable + downsample + stem
    # a plain torchvision-style state dict (no metadata) loads strictly
    plain = {k: v for k, v in net.state_dict().items() if k not in extra}
    net2 = resnet.resnet50()
    net2.load_state_dict(plain)


def test_r50_assignment_matches_published_totals():
    """2448 x 8-bit, 17133 x 6-bit, 3075 x 4-bit, 16,622,232 params."""
    import resnet
    from smpq import assignments
    asg = assignments.load_assignment("r50_mixed")
    assert assignments.bit_histogram(asg) == {4: 3075, 6: 17133, 8: 2448}
    net = resnet.resnet50()
    total = 0.0
    for ln, cn, ch in zip(asg["lnum"], asg["cnum"], asg["chain"]):
        conv = assignments.conv_for_lnum(net, int(ln))
        numel = conv.weight[cn].numel()
        prev = 32
        for b in ch:
            if b:
                total += numel * ((32 - b) / 32 - (32 - prev) / 32)
                prev = b
    assert int(round(total)) == 16622232
    chains = {}
    for ch in asg["chain"]:
        t = tuple(int(b) for b in ch if b)
        chains[t] = chains.get(t, 0) + 1
    assert chains == {(6,): 17133, (4,): 2938, (8,): 2448, (8, 4): 80, (6, 4): 57}


def test_other_assignments():
    from smpq import assignments
    assert assignments.bit_histogram("r18_u8") == {8: 3840}
    assert assignments.bit_histogram("r34_4bit") == {4: 5668, 6: 909, 8: 975}


def test_lnum_binding():
    import resnet
    from smpq import assignments
    net = resnet.resnet34()
    convs = assignments.addressable_convs(net)
    assert len(convs) == 32
    for ln in range(1, 33):
        assert assignments.conv_for_lnum(net, ln) is convs[ln - 1]
    net = resnet.resnet50()
    assert assignments.conv_for_lnum(net, 48) is net.layer4[2].conv3
    assert assignments.conv_for_lnum(net, 25) is net.layer3[1].conv1
