#!/usr/bin/env python3
"""Why does an evaluation pass recapture its graphs? Runs functions.evaluate_acc_loss_softmax three
times over the same device batches and prints, per set_calibration call, which part of its
keep-the-installed-calibration test failed, and per evaluation the engine counters. Diagnostics."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
import functions  # noqa: E402
import resnet  # noqa: E402
from smpq import assignments, engine, stats  # noqa: E402

orig = engine.set_calibration


def traced(model, c, widen=True):
    old = getattr(model, "_smpq_ranges", None)
    sig = engine._signature(model)
    if old is not None:
        maxima = c.maxima.cpu().tolist()
        ranges = {k: max(v, 1e-30) * engine.HEADROOM for k, v in zip(c.keys, maxima)}
        diff = [k for k in ranges if old[0].get(k) != ranges[k]]
        sdiff = [i for i, (a, b) in enumerate(zip(old[1][2], sig[2])) if a != b] if old[1] != sig else []
        print("set_calibration: widen=%s changed=%s sig_equal=%s (differing param/buffer entries %s, convs equal %s) "
              "ranges_equal=%s (%d differ)" % (widen, c.changed, old[1] == sig, sdiff[:5], old[1][3] == sig[3],
                                             not diff, len(diff)), flush=True)
    before = id(getattr(model, "_smpq_ranges", None))
    orig(model, c, widen)
    print("  calibration object kept:", before == id(model._smpq_ranges), flush=True)


engine.set_calibration = traced
dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = resnet.resnet50().to(dev).eval()
assignments.apply_assignment(net, "r50_mixed")
g = torch.Generator().manual_seed(5)
batches = [(torch.randn(256, 3, 224, 224, generator=g).to(dev), torch.randint(0, 1000, (256,), generator=g).to(dev))
           for _ in range(8)]
keys = ("calibrations", "overflow_reruns", "stale_reruns", "graph_captures", "graph_replays", "repack")
for it in range(3):
    s0 = {k: stats[k] for k in keys}
    functions.evaluate_acc_loss_softmax(net, dev, batches)
    torch.cuda.synchronize()
    print("evaluation %d:" % it, {k: stats[k] - s0[k] for k in keys}, flush=True)
