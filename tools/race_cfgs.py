#!/usr/bin/env python3
"""Diagnostics: run one dynamic-mode (fp32 output + per-image max) and one static-mode (limb planes)
quantized conv per tile config REPS times on R18 3x3 shapes and report configs whose outputs are not
bitwise reproducible (an intra-kernel race or hazard shows up as intermittent mismatches).
usage: python tools/race_cfgs.py [reps] [batch]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"), REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from smpq import ops  # noqa: E402
from test_gpu import make_layer  # noqa: E402

gpu = torch.device("cuda")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
for cin, cout, k, s, h in [(64, 64, 3, 1, 56), (128, 128, 3, 1, 28), (256, 256, 3, 1, 14), (512, 512, 3, 1, 7),
                           (64, 128, 3, 2, 56)]:
    wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin + 3 * cout)
    g = torch.Generator().manual_seed(5)
    x = torch.relu(torch.randn(B, h, h, cin, generator=g)).to(gpu)
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, 3)
    shift = torch.linspace(-1, 1, cout, device=gpu)
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    bad_cfgs = []
    for c in ops.tile_configs():
        if not ops._tile_fits(c, 3, 1, False, cout, cin, k):
            continue
        base = None
        bad = 0
        for r in range(reps):
            yam = torch.zeros(B, device=gpu)
            y = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=True, y_absmax=yam, tile_cfg=c)
            _, q = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=True, tile_cfg=c,
                                emit_range=8.0, overflow=ovf, want_f32=False)
            out = (y.clone(), yam.clone(), q.clone())
            if base is None:
                base = out
            elif not all(torch.equal(u, v) for u, v in zip(out, base)):
                bad += 1
        if bad:
            bad_cfgs.append((c, bad))
    print("shape", (cin, cout, k, s, h), "B", B, "non-reproducible configs (cfg, runs):", bad_cfgs, flush=True)
