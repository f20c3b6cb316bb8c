#!/usr/bin/env python3
"""Time single static-range quantized-conv launches of the R50 shapes (B=256, L=3) for chosen
tile configs, and check that every config's output limb planes equal those of the C-ABI default
(bit for bit). Diagnostics only.

    python tools/tile_bench.py [cfg,cfg,...|all] [shape-substring]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from smpq import ops  # noqa: E402

L, B = 3, int(os.environ.get("TB_BATCH", "256"))
CFGS = None if len(sys.argv) < 2 or sys.argv[1] == "all" else [int(c) for c in sys.argv[1].split(",")]
ONLY = sys.argv[2] if len(sys.argv) > 2 else None
SHAPES = [  # name, cin, cout, k, stride, hin, residual, wlimbs
    ("c1_256_64_56", 256, 64, 1, 1, 56, False, 1),
    ("c2_64_64_56", 64, 64, 3, 1, 56, False, 1),
    ("c3_64_256_56r", 64, 256, 1, 1, 56, True, 1),
    ("c2_128_128_28", 128, 128, 3, 1, 28, False, 1),
    ("c2_128_128_56s2", 128, 128, 3, 2, 56, False, 1),
    ("c1_512_128_28", 512, 128, 1, 1, 28, False, 1),
    ("c3_128_512_28r", 128, 512, 1, 1, 28, True, 1),
    ("c2_256_256_14", 256, 256, 3, 1, 14, False, 1),
    ("c1_1024_256_14", 1024, 256, 1, 1, 14, False, 1),
    ("c3_256_1024_14r", 256, 1024, 1, 1, 14, True, 1),
    ("c2_512_512_7", 512, 512, 3, 1, 7, False, 1),
    ("c1_2048_512_7", 2048, 512, 1, 1, 7, False, 1),
    ("ds_1024_2048_14s2", 1024, 2048, 1, 2, 14, False, 3),
    ("ds_512_1024_28s2", 512, 1024, 1, 2, 28, False, 3),
    ("ds_256_512_56s2", 256, 512, 1, 2, 56, False, 3),
    ("ds_64_256_56", 64, 256, 1, 1, 56, False, 3),
]
dev = torch.device("cuda")
for name, cin, cout, k, s, h, res, wl in SHAPES:
    if ONLY and ONLY not in name:
        continue
    g = torch.Generator(device=dev).manual_seed(0)
    w = torch.randn(cout, cin, k, k, device=dev, generator=g) * 0.05
    if wl == 1:
        step = ops.quantize_channels_(w.reshape(cout, -1), [6] * cout)
        codes, offset, wscale, st = ops.pack_weights_ex(w, step, 1)
    else:
        codes, offset, wscale, st = ops.pack_weights_ex(w, None, wl)
    offset = None
    x = torch.relu(torch.randn(B, h, h, cin, device=dev, generator=g))
    am = ops.act_absmax(x)
    xq = ops.act_quantize(x, am, L)
    ho = (h + 2 * (k // 2) - k) // s + 1
    rq = ops.act_quantize(torch.relu(torch.randn(B, ho, ho, cout, device=dev, generator=g)),
                          torch.full((B,), 4.0, device=dev), L) if res else None
    shift = torch.linspace(-0.1, 0.1, cout, device=dev)
    ovf = torch.zeros(2, dtype=torch.int32, device=dev)
    kw = dict(emit_range=8.0, overflow=ovf, want_f32=False, relu=True)
    if res:
        kw.update(residual_q=rq, residual_range=4.0)
    _, ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, wscale, shift, tile_cfg=-1, **kw)
    out = []
    for c in ops.tile_configs():
        if ops.tile_kind(c) not in (ops.TILE_LDS_DMA, ops.TILE_LDS_DMA_K128):
            continue
        if not ops._tile_fits(c, L, wl, cout, cin, k) or (CFGS is not None and c not in CFGS):
            continue
        try:
            _, y = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, wscale, shift, tile_cfg=c, **kw)
        except Exception as e:  # noqa: BLE001
            out.append("cfg%d: %s" % (c, str(e)[:40]))
            continue
        same = torch.equal(y, ref)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(10):
            ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, wscale, shift, tile_cfg=c, **kw)
        ev[1].record()
        torch.cuda.synchronize()
        t = ev[0].elapsed_time(ev[1]) / 10 * 1e3
        out.append("cfg%d %6.1fus%s" % (c, t, "" if same else " MISMATCH"))
    print("%-18s | %s" % (name, " | ".join(out)), flush=True)
