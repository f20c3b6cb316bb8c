#!/usr/bin/env python3
"""Diagnostics: repeat tests/test_gpu.py::test_graph_replay_matches_eager's sequence N times in
one process and report which outputs differ (eager vs graph replay, per image, max |diff|).
usage: python tools/repro_graph.py [N]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"), REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

if os.environ.get("SMPQ_LIB"):  # an older diagnostic build: bind only the symbols it has
    import ctypes
    from smpq import _lib
    have = ctypes.CDLL(os.environ["SMPQ_LIB"])
    for k in list(_lib._PROTOS):
        if not hasattr(have, k):
            del _lib._PROTOS[k]
else:
    __graft_entry__.build()
from test_gpu import build_model  # noqa: E402
from smpq import engine, stats  # noqa: E402

gpu = torch.device("cuda:0")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for it in range(N):
    net = build_model(gpu, "resnet50", "r50_mixed")
    x = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(14)).to(gpu)
    x2 = torch.randn(6, 3, 224, 224, generator=torch.Generator().manual_seed(15)).to(gpu)
    with torch.no_grad():
        engine.USE_GRAPH[0] = False
        net(x)
        e1, e2 = net(x), net(x2)
        e2b = net(x2)
        engine.USE_GRAPH[0] = True
        g1 = net(x)
        g2 = net(x2)
        g3 = net(x)
        g4 = net(x2)
    d = lambda a, b: [round(v, 5) for v in (a - b).abs().amax(1).tolist()]  # noqa: E731
    print("iter", it, "overflow_reruns", stats.get("overflow_reruns"), flush=True)
    print("  e2b-e2", d(e2b, e2), "g1-e1", d(g1, e1), "g2-e2", d(g2, e2), "g3-e1", d(g3, e1), "g4-e2", d(g4, e2),
          flush=True)
