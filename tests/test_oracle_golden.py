"""Pin the oracle to the reference: golden vectors produced by importing the reference itself
(tests/golden/make_golden.py). CPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import eval_ref, forward_ref, quant_ref


def _kat():
    return np.load(os.path.join(GOLDEN, "quant_kat.npz"), allow_pickle=False)


def kat_cases():
    z = _kat()
    off = z["offsets"]
    for i in range(len(z["kinds"])):
        chain = [int(b) for b in z["chain"][i] if b]
        yield str(z["kinds"][i]), chain, z["x"][off[i]:off[i + 1]], z["y"][off[i]:off[i + 1]]


def device_kat_cases():
    """The KAT inputs quantized by torch ON THE GPU (tests/golden/make_device_kat.py, run on an
    MI355X) plus extra channels where the GPU and CPU results differ: (kind, chain, x, y_device)."""
    d = np.load(os.path.join(GOLDEN, "quant_kat_device.npz"), allow_pickle=False)
    z = _kat()
    off = z["offsets"]
    for i in range(len(z["kinds"])):
        chain = [int(b) for b in z["chain"][i] if b]
        yield str(z["kinds"][i]), chain, z["x"][off[i]:off[i + 1]], d["y_device"][off[i]:off[i + 1]]
    eo = d["ex_offsets"]
    for i in range(len(d["ex_bits"])):
        yield "gpu-differs", [int(d["ex_bits"][i])], d["ex_x"][eo[i]:eo[i + 1]], d["ex_y_device"][eo[i]:eo[i + 1]]


def test_device_kat_differs_from_cpu_somewhere():
    # the device fixture is informative: torch on the GPU rounds some channels differently
    d = np.load(os.path.join(GOLDEN, "quant_kat_device.npz"), allow_pickle=False)
    assert int(d["differs_from_cpu_cases"]) >= 1 and len(d["ex_bits"]) >= 1
    assert not np.array_equal(d["ex_y_device"], d["ex_y_cpu"])


def test_quant_oracle_device_semantics_vs_torch_gpu():
    n = 0
    for kind, chain, x, y in device_kat_cases():
        out = quant_ref.apply_chain(x, chain, semantics="device")
        assert np.array_equal(out.view(np.uint32), y.view(np.uint32)), (kind, chain)
        n += 1
    assert n >= 70


def test_quant_oracle_bitexact_vs_reference():
    n = 0
    for kind, chain, x, y in kat_cases():
        out = quant_ref.apply_chain(x, chain)
        assert np.array_equal(out.view(np.uint32), y.view(np.uint32)), (kind, chain)
        n += 1
    assert n >= 60


def test_quant_oracle_tie_case_five_levels():
    # functions.py:41 ties: 2-bit can produce 2^b + 1 = 5 levels
    out = quant_ref.quantize_wgt(np.array([-1, -.5, 0, .5, 1, .3], np.float32), 2)
    np.testing.assert_allclose(out, [-4 / 3, -2 / 3, 0, 2 / 3, 4 / 3, 0], rtol=1e-6)
    assert len(np.unique(out)) == 5


def test_quant_oracle_constant_channel_raises():
    assert bool(_kat()["const_raises"])
    with pytest.raises(ZeroDivisionError):
        quant_ref.quantize_wgt(np.full(9, 0.25, np.float32), 8)


def test_quant_codes_reconstruct():
    for kind, chain, x, y in kat_cases():
        if len(chain) != 1:
            continue
        m, s = quant_ref.quantize_codes(x, chain[0])
        assert np.array_equal((m.astype(np.float32) * s).view(np.uint32), y.view(np.uint32))
        assert m.max() - m.min() <= 2 ** chain[0]


def _goldens():
    return np.load(os.path.join(GOLDEN, "model_goldens.npz"), allow_pickle=False)


def seeded_state(arch, assign=None, cal=None):
    """State dict (numpy) of the seeded model with the oracle quantizer applied."""
    import resnet
    from smpq import assignments
    torch.manual_seed(0)
    net = getattr(resnet, arch)()
    sd = {k: v.numpy().copy() for k, v in net.state_dict().items()}
    if assign is not None:
        asg = assignments.load_assignment(assign)
        names = {id(m): n for n, m in net.named_modules()}
        for ln, cn, ch in zip(asg["lnum"], asg["cnum"], asg["chain"]):
            conv = assignments.conv_for_lnum(net, int(ln))
            key = names[id(conv)] + ".weight"
            sd[key][cn] = quant_ref.apply_chain(sd[key][cn], [int(b) for b in ch if b])
    if cal is not None:
        g = _goldens()
        pref = cal + "/bn/"
        for k in g.files:
            if k.startswith(pref):
                sd[k[len(pref):]] = g[k]
    return sd


@pytest.mark.parametrize("case,arch,assign,batch", [("r18_fp32", "resnet18", None, 2), ("r18_u8", "resnet18", "r18_u8", 2),
                                                    ("r18_u8_b1", "resnet18", "r18_u8", 1)])
def test_forward_oracle_vs_reference_logits(case, arch, assign, batch):
    g = _goldens()
    sd = seeded_state(arch, assign)
    for k in g.files:
        if k.startswith(case + "/qsum/"):
            w = sd[k[len(case + "/qsum/"):]].astype(np.float64)
            np.testing.assert_allclose([w.sum(), np.abs(w).sum()], g[k], rtol=1e-9, atol=1e-9)
    x = torch.randn(batch, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    np.testing.assert_allclose([x.double().sum().item(), x.double().abs().sum().item()], g[case + "/xsum"], rtol=1e-12)
    out = forward_ref.resnet_forward(arch, sd, x.numpy())
    ref = g[case + "/logits"]
    assert np.abs(out - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-5
    assert (out.argmax(1) == ref.argmax(1)).all()


def test_forward_oracle_r50_mixed_vs_reference_logits():
    g = _goldens()
    sd = seeded_state("resnet50", "r50_mixed")
    x = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    out = forward_ref.resnet_forward("resnet50", sd, x.numpy())
    ref = g["r50_mixed/logits"]
    assert np.abs(out - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-5


def test_torch_oracle_reproduces_reference_logits():
    from oracle import torch_ref
    g = _goldens()
    for case, arch, assign in (("r18_u8", "resnet18", "r18_u8"), ("r50_mixed", "resnet50", "r50_mixed")):
        sd = {k: torch.from_numpy(v) for k, v in seeded_state(arch, assign).items()}
        x = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(1))
        out = torch_ref.resnet_forward(arch, sd, x).numpy()
        ref = g[case + "/logits"]
        assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()


@pytest.mark.parametrize("case,arch,assign", [("r18_u8_cal", "resnet18", "r18_u8"),
                                              ("r34_4bit_cal", "resnet34", "r34_4bit"),
                                              ("r50_mixed_cal", "resnet50", "r50_mixed")])
def test_torch_oracle_reproduces_recalibrated_reference_logits(case, arch, assign):
    """The oracle the full-size GPU parity tests compare against (oracle/torch_ref.py) reproduces
    the reference's own logits on the BN-recalibrated parity models of all three bench archs."""
    from oracle import torch_ref
    g = _goldens()
    sd = {k: torch.from_numpy(v) for k, v in seeded_state(arch, assign, cal=case).items()}
    ref = g[case + "/logits"]
    x = torch.randn(ref.shape[0], 3, 224, 224, generator=torch.Generator().manual_seed(1))
    np.testing.assert_allclose([x.double().sum().item(), x.double().abs().sum().item()], g[case + "/xsum"], rtol=1e-12)
    out = torch_ref.resnet_forward(arch, sd, x).numpy()
    assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()
    assert (out.argmax(1) == ref.argmax(1)).all()


def _eval_golden():
    z = np.load(os.path.join(GOLDEN, "eval_golden.npz"), allow_pickle=False)
    cuts = np.cumsum([0] + list(z["sizes"]))
    split = lambda a: [a[cuts[i]:cuts[i + 1]] for i in range(len(cuts) - 1)]  # noqa: E731
    return z, split


def test_eval_oracle_vs_reference():
    # functions.py:84-149 run by the reference itself on seeded logits (ragged batch, tied row)
    z, split = _eval_golden()
    batches = list(zip(split(z["logits_a"]), split(z["labels"])))
    acc, loss, outs = eval_ref.evaluate_acc_loss_softmax(batches)
    assert abs(acc - float(z["acc_a"])) < 1e-7  # the reference divides in fp32 (functions.py:125)
    assert abs(loss - float(z["loss_a"])) < 1e-5 * abs(float(z["loss_a"]))
    np.testing.assert_allclose(np.concatenate(outs), z["softmax_a"], rtol=1e-5, atol=1e-9)
    acc_b, loss_b, outs_b = eval_ref.evaluate_acc_loss_softmax(list(zip(split(z["logits_b"]), split(z["labels"]))))
    assert abs(acc_b - float(z["acc_b"])) < 1e-7 and abs(loss_b - float(z["loss_b"])) < 1e-5 * abs(float(z["loss_b"]))
    kl = eval_ref.kldiv(split(z["softmax_a"]), split(z["softmax_b"]))
    assert abs(kl - float(z["kl"])) < 1e-5 * abs(float(z["kl"]))
