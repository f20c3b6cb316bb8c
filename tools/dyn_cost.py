#!/usr/bin/env python3
"""Per-forward cost of the dynamic-range mode's staleness guarantee: the host
signature walk over every parameter / buffer, the device content fingerprint of the weights, BN
tensors and quantization metadata (csrc/fingerprint.hip), and the one host sync that reads its
flag — measured beside the whole dynamic forward of the bench model (R50 mixed, B=256, L=3).
Writes one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
import resnet  # noqa: E402
from smpq import assignments, engine  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
net = resnet.resnet50().to(dev).eval()
assignments.apply_assignment(net, "r50_mixed")
engine.set_range_mode("dynamic")
x = torch.randn(256, 3, 224, 224, device=dev)
with torch.no_grad():
    for _ in range(3):
        net(x)
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        net(x)
    torch.cuda.synchronize()
    fwd_ms = (time.perf_counter() - t0) / n * 1e3
    # the pieces, alone
    t0 = time.perf_counter()
    for _ in range(100):
        engine._signature(net)
    sig_ms = (time.perf_counter() - t0) / 100 * 1e3
    fp = net._smpq_dyn[1]
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fp.check(flag)
    e1.record()
    torch.cuda.synchronize()
    check_ms = e0.elapsed_time(e1) / 20
    t0 = time.perf_counter()
    for _ in range(100):
        int(flag.item())
    sync_ms = (time.perf_counter() - t0) / 100 * 1e3
out = {"model": "R50 mixed 8/6/4, B=256, L=3, dynamic ranges", "forward_ms": round(fwd_ms, 3),
       "host_signature_walk_ms": round(sig_ms, 3), "device_fingerprint_check_ms": round(check_ms, 3),
       "flag_host_sync_ms": round(sync_ms, 4),
       "guarantee_share_of_forward": round((sig_ms + check_ms + sync_ms) / fwd_ms, 4)}
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
print(json.dumps(out))
