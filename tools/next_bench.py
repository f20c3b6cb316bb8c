#!/usr/bin/env python3
"""Time the fused conv3 + next conv1 launch (ops.conv2d_q_next) against the two separate autotuned
launches on the R50 pair shapes (B=256, L=3), per fused tile; SMPQ_NX_ABLATE=1/2 drops the next
conv's stores / MFMAs (diagnostic builds of the timing only). Diagnostics only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from smpq import ops  # noqa: E402

B = int(os.environ.get("NB_BATCH", "256"))
dev = torch.device("cuda")
PAIRS = [("l1_c3+c1", 64, 256, 64, 56), ("l1->l2", 64, 256, 128, 56), ("l2_c3+c1", 128, 512, 128, 28),
         ("l2->l3", 128, 512, 256, 28)]


def timeit(fn, reps=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, cmid, cout, ncout, h in PAIRS:
    g = torch.Generator(device=dev).manual_seed(0)
    w3 = torch.randn(cout, cmid, 1, 1, device=dev, generator=g) * 0.05
    w1 = torch.randn(ncout, cout, 1, 1, device=dev, generator=g) * 0.05
    s3 = ops.quantize_channels_(w3.reshape(cout, -1), [6] * cout)
    s1 = ops.quantize_channels_(w1.reshape(ncout, -1), [6] * ncout)
    c3, _, ws3, _ = ops.pack_weights_ex(w3, s3, 1)
    c1, _, ws1, _ = ops.pack_weights_ex(w1, s1, 1)
    x = torch.relu(torch.randn(B, h, h, cmid, device=dev, generator=g))
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    rq = ops.act_quantize(torch.relu(torch.randn(B, h, h, cout, device=dev, generator=g)),
                          torch.full((B,), 4.0, device=dev), 3)
    sh3 = torch.zeros(cout, device=dev)
    sh1 = torch.zeros(ncout, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    ram = torch.full((B,), 8.0, device=dev)
    kw3 = dict(relu=True, residual_q=rq, residual_range=4.0, emit_range=8.0, overflow=ovf, want_f32=False)

    def sep():
        _, q3 = ops.tuned_conv2d_q(xq, am, c3, None, 1, 1, 1, 0, ws3, sh3, **kw3)
        ops.tuned_conv2d_q(q3, ram, c1, None, 1, 1, 1, 0, ws1, sh1, relu=True, emit_range=8.0, overflow=ovf,
                           want_f32=False)

    def one(which):
        _, q3 = ops.tuned_conv2d_q(xq, am, c3, None, 1, 1, 1, 0, ws3, sh3, **kw3)
        if which == 2:
            ops.tuned_conv2d_q(q3, ram, c1, None, 1, 1, 1, 0, ws1, sh1, relu=True, emit_range=8.0, overflow=ovf,
                               want_f32=False)

    t3 = timeit(lambda: ops.tuned_conv2d_q(xq, am, c3, None, 1, 1, 1, 0, ws3, sh3, **kw3))
    ts = timeit(sep)
    out = ["conv3 %.1f" % t3, "conv3+conv1 separate %.1f" % ts]
    if cout == 256:  # conv3 alone on the fused kernel's 256 x 32 tile (LDS-DMA config 7)
        c7 = min(c for c in ops.tile_configs() if ops.tile_kind(c) == ops.TILE_LDS_DMA) + 7
        out.append("conv3 256x32 %.1f" % timeit(lambda: ops.conv2d_q(xq, am, c3, None, 1, 1, 1, 0, ws3, sh3, tile_cfg=c7,
                                                                     **kw3)))
    for c in ops.next_tile_configs(cmid, cout, 1, ncout):
        t = timeit(lambda: ops.conv2d_q_next(xq, am, c3, None, 1, 1, 1, 0, ws3, sh3, 8.0, ovf, c1, ram, ws1, sh1, 8.0,
                                             residual_q=rq, residual_range=4.0, tile_cfg=c))
        out.append("fused cfg%d %.1f" % (c, t))
    print("%-10s ablate=%s | %s" % (name, os.environ.get("SMPQ_NX_ABLATE", "0"), " | ".join(out)), flush=True)
