#!/usr/bin/env python3
"""Time the fused Bottleneck tail (each tile config) against the two-launch path on the R50
shapes. Diagnostics only. usage: python tools/tail_microbench.py [limbs] [batch]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from smpq import ops  # noqa: E402
from test_gpu import _tail_case  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
OFF = len(sys.argv) > 3 and sys.argv[3] == "offsets"
dev = torch.device("cuda")


def timeit(fn, reps=10):
    fn()
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for h, cmid, stride in ((56, 64, 1), (56, 128, 2), (28, 128, 1), (14, 256, 1), (7, 512, 1)):
    xq, am, c2, c3, resq, rr, ho = _tail_case(dev, B, h, cmid, stride, L, 7, offsets=OFF)
    ovf = torch.zeros(2, dtype=torch.int32, device=dev)
    r2, r3 = 40.0, 60.0
    n = B
    ra = torch.full((n,), r2, device=dev)

    def unfused():
        _, t2 = ops.tuned_conv2d_q(xq, am, c2[0], c2[1], 3, 3, stride, 1, c2[2], c2[3], relu=True, emit_range=r2,
                                   overflow=ovf, want_f32=False)
        ops.tuned_conv2d_q(t2, ra, c3[0], c3[1], 1, 1, 1, 0, c3[2], c3[3], relu=True, emit_range=r3, overflow=ovf,
                           want_f32=False, residual_q=resq, residual_range=rr)

    def conv2_only():
        ops.tuned_conv2d_q(xq, am, c2[0], c2[1], 3, 3, stride, 1, c2[2], c2[3], relu=True, emit_range=r2,
                           overflow=ovf, want_f32=False)
    out = ["unfused %.1f (conv2 %.1f)" % (timeit(unfused), timeit(conv2_only))]
    for cfg in ops.tail_configs():
        if not ops.tail_supported(cfg, cmid, 4 * cmid, 3, L):
            continue
        t = timeit(lambda: ops.bottleneck_tail_q(xq, am, c2[0], c2[1], 3, stride, 1, c2[2], c2[3], r2, c3[0], c3[1],
                                                 c3[2], c3[3], resq, rr, r3, ovf, cfg))
        out.append("cfg%d %.1f" % (cfg, t))
    print("h%d cmid%d s%d B%d L%d: %s" % (h, cmid, stride, B, L, " | ".join(out)), flush=True)
