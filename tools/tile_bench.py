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
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from smpq import ops  # noqa: E402

L, B = 3, int(os.environ.get("TB_BATCH", "256"))
CFGS = None if len(sys.argv) < 2 or sys.argv[1] == "all" else [int(c) for c in sys.argv[1].split(",")]
ONLY = sys.argv[2] if len(sys.argv) > 2 else None
from r50_shapes import SHAPES  # noqa: E402
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
    # wide output range: nothing overflows (an overflowing launch also times its flag atomics)
    kw = dict(emit_range=1000.0, overflow=ovf, want_f32=False, relu=wl == 1)  # the downsamples: no ReLU
    if res:
        kw.update(residual_q=rq, residual_range=4.0)
    _, ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, wscale, shift, tile_cfg=-1, **kw)
    out = []
    for c in ops.tile_configs():
        if ops.tile_kind(c) not in (ops.TILE_LDS_DMA, ops.TILE_LDS_DMA_K128, ops.TILE_HALO3X3, ops.TILE_RESIDENT1X1):
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
