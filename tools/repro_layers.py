#!/usr/bin/env python3
"""Diagnostics: run the static eager forward of x, then of x2, then of x again (no graphs), record
every quantized conv's limb-plane / fp32 output and maxpool output, and print the first launches
whose outputs differ between the two runs on x (state-dependent results = a race or a read of
uninitialized memory). usage: python tools/repro_layers.py [iterations]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"), REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from test_gpu import build_model  # noqa: E402
from smpq import engine, ops  # noqa: E402

gpu = torch.device("cuda:0")
REC = []
_conv = ops.conv2d_q
_stem = ops.stem_conv_s2d
_pool = ops.maxpool_limbs


def conv_rec(*a, **k):
    r = _conv(*a, **k)
    outs = r if isinstance(r, tuple) else (r,)
    xq = a[0]
    REC.append(("conv", tuple(xq.shape), a[2].shape if a[2] is not None else None, k.get("tile_cfg"),
                [o.clone() if o is not None else None for o in outs]))
    return r


def stem_rec(*a, **k):
    r = _stem(*a, **k)
    outs = r if isinstance(r, tuple) else (r,)
    REC.append(("stem", None, None, k.get("tile_cfg"), [o.clone() if o is not None else None for o in outs]))
    return r


def pool_rec(*a, **k):
    r = _pool(*a, **k)
    REC.append(("pool", tuple(a[0].shape), None, None, [r.clone()]))
    return r


ops.conv2d_q = conv_rec
ops.stem_conv_s2d = stem_rec
ops.maxpool_limbs = pool_rec
engine.USE_GRAPH[0] = False
N = int(sys.argv[1]) if len(sys.argv) > 1 else 3
MODE = sys.argv[2] if len(sys.argv) > 2 else "static"   # "dynamic-first": first call (autotuning) vs second
for it in range(N):
    if MODE in ("dynamic-first", "dynamic-pair"):
        engine.set_range_mode("dynamic")
        if MODE == "dynamic-first":
            ops._TUNED.clear()
        net = build_model(gpu, "resnet18", "r18_u8")
        x = torch.randn(64, 3, 224, 224, generator=torch.Generator().manual_seed(11)).to(gpu)
        with torch.no_grad():
            if MODE == "dynamic-pair":
                net(x)
            REC.clear()
            e1 = net(x)
            r1 = list(REC)
            REC.clear()
            e3 = net(x)
            r3 = list(REC)
        engine.set_range_mode("static")
    else:
        net = build_model(gpu, "resnet50", "r50_mixed")
        x = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(14)).to(gpu)
        x2 = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(15)).to(gpu)
        with torch.no_grad():
            net(x)
            net(x)  # autotune outside the recorded runs
            REC.clear()
            e1 = net(x)
            r1 = list(REC)
            net(x2)
            REC.clear()
            e3 = net(x)
            r3 = list(REC)
    torch.cuda.synchronize()
    diff = (e1 - e3).abs().amax(1).tolist()
    print("iter", it, "logits diff per image", [round(v, 5) for v in diff], "launches", len(r1), len(r3), flush=True)
    shown = 0
    for i, (a, b) in enumerate(zip(r1, r3)):
        for t, (u, v) in enumerate(zip(a[4], b[4])):
            if u is None or torch.equal(u, v):
                continue
            bad = (u != v)
            idx = bad.nonzero()
            print("  launch %d %s xq=%s w=%s cfg=%s out%d: %d elements differ, first %s, shape %s" %
                  (i, a[0], a[1], tuple(a[2]) if a[2] is not None else None, a[3], t, int(bad.sum()),
                   idx[:4].tolist(), tuple(u.shape)), flush=True)
            shown += 1
        if shown >= 6:
            break
