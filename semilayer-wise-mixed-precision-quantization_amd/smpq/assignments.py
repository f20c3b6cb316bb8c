"""Per-channel bit assignments (the semilayer search's output) and their application.

Files in ``smpq/data/assign_*.npz`` (made by tests/golden/make_golden.py from the reference's
own data files):
  * ``r50_mixed``  — the published ResNet-50 8/6/4-bit result, reconstructed from
    dataset/resnet50_deltaloss.csv + output/resnet50ImageNetq864bit_mixedprecision_accs.csv
    (reproduces the published 16,622,232 reduced parameters);
  * ``r18_u8``     — ResNet-18 uniform 8-bit on the 16 addressable convs;
  * ``r34_4bit``   — ResNet-34 4-bit-dominant rule on dataset/resnet34_deltaloss.csv
    (SURVEY.md 8(d) C5).
Each row: (lnum, cnum 0-based, chain of up to 3 bits applied in order, 0 = none).

lnum -> conv binding: R50 lnum = 3*(global block) + {1,2,3} -> conv{1,2,3}
(resnet50_main.py:81-136,189-197); R18/R34 odd -> conv1, even -> conv2 in block order
(resnet18_main.py:86-115; for R34 the intended [3,4,6,3] map, not the copy-pasted R18 map
at resnet34_main.py:86-109).
"""
import os

import numpy as np

from .quant import quantize_layer_

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def load_assignment(name):
    z = np.load(os.path.join(DATA, "assign_%s.npz" % name), allow_pickle=False)
    return {"arch": str(z["arch"]), "lnum": z["lnum"].astype(np.int64),
            "cnum": z["cnum"].astype(np.int64), "chain": z["chain"].astype(np.int64)}


def blocks_of(net):
    return [b for layer in (net.layer1, net.layer2, net.layer3, net.layer4) for b in layer]


def conv_for_lnum(net, lnum):
    blocks = blocks_of(net)
    if hasattr(blocks[0], "conv3"):
        b = blocks[(lnum - 1) // 3]
        return (b.conv1, b.conv2, b.conv3)[(lnum - 1) % 3]
    b = blocks[(lnum - 1) // 2]
    return b.conv1 if lnum % 2 == 1 else b.conv2


def addressable_convs(net):
    """Quantizable convs in lnum order (16 / 32 / 48 for R18 / R34 / R50)."""
    out = []
    for b in blocks_of(net):
        out += [b.conv1, b.conv2] + ([b.conv3] if hasattr(b, "conv3") else [])
    return out


def apply_assignment(net, assign, semantics=None):
    """Fake-quantize ``net`` per channel chain; one launch per (conv, chain step). ``semantics``:
    the rounding of functions.py:41 (ops.set_quant_semantics; None = the process setting)."""
    if isinstance(assign, str):
        assign = load_assignment(assign)
    lnum, cnum, chain = assign["lnum"], assign["cnum"], assign["chain"]
    by_conv = {}
    for ln in np.unique(lnum):
        by_conv[int(ln)] = np.nonzero(lnum == ln)[0]
    for step in range(chain.shape[1]):
        for ln, rows in by_conv.items():
            conv = conv_for_lnum(net, ln)
            bits = np.zeros(conv.out_channels, dtype=np.int64)
            bits[cnum[rows]] = chain[rows, step]
            if (bits > 0).any():
                quantize_layer_(conv, bits, semantics=semantics)
    return net


def bit_histogram(assign):
    if isinstance(assign, str):
        assign = load_assignment(assign)
    final = np.array([c[c > 0][-1] if (c > 0).any() else 32 for c in assign["chain"]])
    return {int(b): int((final == b).sum()) for b in np.unique(final)}
