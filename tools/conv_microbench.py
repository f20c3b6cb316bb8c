#!/usr/bin/env python3
"""Time single quantized-conv launches of representative R50 shapes (B=256) per tile config.
Diagnostics only. usage: python tools/conv_microbench.py [limbs] [static|dynamic] [shape-substr] [cfg,...]
With SMPQ_ABLATE set (see conv.hip) the numbers are ablations (wrong results)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from smpq import ops  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 3
static = (sys.argv[2] if len(sys.argv) > 2 else "static") == "static"
B = 256
ONLY = sys.argv[3] if len(sys.argv) > 3 else None
CFGS = [int(c) for c in sys.argv[4].split(",")] if len(sys.argv) > 4 else None
SHAPES = [  # name, cin, cout, k, stride, hin, residual
    ("c1_256_64_56", 256, 64, 1, 1, 56, False),
    ("c2_64_64_56", 64, 64, 3, 1, 56, False),
    ("c3_64_256_56", 64, 256, 1, 1, 56, True),
    ("ds_64_256_56", 64, 256, 1, 1, 56, False),
    ("c2_256_256_14", 256, 256, 3, 1, 14, False),
    ("c2_128_128_28", 128, 128, 3, 1, 28, False),
    ("c2_512_512_7", 512, 512, 3, 1, 7, False),
    ("c1_2048_512_7", 2048, 512, 1, 1, 7, False),
    ("c3_256_1024_14", 256, 1024, 1, 1, 14, True),
    ("c1_1024_256_14", 1024, 256, 1, 1, 14, False),
    ("c1_512_256_28", 512, 256, 1, 1, 28, False),
    ("c1_512_128_28", 512, 128, 1, 1, 28, False),
    ("c3_128_512_28", 128, 512, 1, 1, 28, True),
    ("c1_1024_512_14", 1024, 512, 1, 1, 14, False),
    ("c3_512_2048_7", 512, 2048, 1, 1, 7, True),
]
dev = torch.device("cuda")
for name, cin, cout, k, s, h, res in SHAPES:
    if ONLY and ONLY not in name:
        continue
    g = torch.Generator(device=dev).manual_seed(0)
    w = torch.randn(cout, cin, k, k, device=dev, generator=g) * 0.05
    step = ops.quantize_channels_(w.reshape(cout, -1), [6] * cout)
    codes, offset, wscale, st = ops.pack_weights_ex(w, step, 1)
    x = torch.relu(torch.randn(B, h, h, cin, device=dev, generator=g))
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, L)
    ho = (h + 2 * (k // 2) - k) // s + 1
    rq = ops.act_quantize(torch.relu(torch.randn(B, ho, ho, cout, device=dev, generator=g)),
                          torch.full((B,), 4.0, device=dev), L) if res else None
    shift = torch.zeros(cout, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    ops_n = 2 * B * ho * ho * cout * cin * k * k
    byt = B * h * h * cin * L + B * ho * ho * cout * L * (2 if res else 1)
    out = []
    for c in ops.tile_configs():
        if not ops._tile_fits(c, L, 1, cout, cin, k) or (CFGS is not None and c not in CFGS):
            continue
        kw = dict(emit_range=8.0, overflow=ovf, want_f32=False, relu=True) if static else {}
        if res:
            kw.update(residual_q=rq, residual_range=4.0) if static else kw.update(
                residual=torch.zeros(B, ho, ho, cout, device=dev))
        try:
            for _ in range(2):
                ops.conv2d_q(xq, am, codes, None, k, k, s, k // 2, wscale, shift, tile_cfg=c, **kw)
        except Exception:  # the tile family does not take this shape
            continue
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(10):
            ops.conv2d_q(xq, am, codes, None, k, k, s, k // 2, wscale, shift, tile_cfg=c, **kw)
        ev[1].record()
        torch.cuda.synchronize()
        t = ev[0].elapsed_time(ev[1]) / 10 * 1e3
        out.append("cfg%d %7.1fus %5.0fTOP/s %5.2fTB/s" % (c, t, ops_n / t / 1e6, byt / t / 1e6))
    print("%-16s L=%d %s | %s" % (name, L, "static" if static else "dynamic", " | ".join(out)), flush=True)
