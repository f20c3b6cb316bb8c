#!/usr/bin/env python3
"""Per-launch time of single static-range quantized-conv launches of the R50 shapes against the
batch size (L=3), best tile per (shape, batch), launches replayed from a HIP graph so that host
overhead is out of the timing. A launch whose time does not fall with the batch is bound by the
serial chain of one block (latency), not by a chip-wide throughput. Diagnostics only.

    python tools/batch_scaling.py [shape-substring] [batches, default 32,64,128,256]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from smpq import _lib, ops  # noqa: E402

sys.path.insert(0, os.path.join(REPO, "tools"))
from r50_shapes import SHAPES  # noqa: E402

L = 3
ONLY = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "all" else None
BATCHES = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "32,64,128,256").split(",")]
CFGS = [int(c) for c in os.environ.get("BS_CFGS", "").split(",") if c.strip()] or None
dev = torch.device("cuda")


def timed(fn, reps=10, rounds=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


lib = _lib.load()
for name, cin, cout, k, s, h, res, wl in SHAPES:
    if ONLY and ONLY not in name:
        continue
    row = []
    for B in BATCHES:
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
        best = None
        best_kind = {}
        for c in ops.tile_configs():
            if ops.tile_kind(c) not in (ops.TILE_LDS_DMA, ops.TILE_LDS_DMA_K128, ops.TILE_HALO3X3):
                continue
            if not ops._tile_fits(c, L, wl, cout, cin, k) or (CFGS is not None and c not in CFGS):
                continue
            try:
                t = timed(lambda: ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, wscale, shift, tile_cfg=c, **kw))
            except Exception:  # noqa: BLE001
                continue
            if best is None or t < best[0]:
                best = (t, c)
            kd = ops.tile_kind(c)
            if kd not in best_kind or t < best_kind[kd][0]:
                best_kind[kd] = (t, c)
        bm, bn, thr = ops.tile_configs()[best[1]]  # BM pixels x BN channels
        blocks = ((B * ho * ho + bm - 1) // bm) * ((cout + bn - 1) // bn)
        kinds = " ".join("k%d:%.1f(c%d)" % (kd, tk, ck) for kd, (tk, ck) in sorted(best_kind.items()))
        row.append("B=%-3d %7.1fus %5.3fus/img cfg%-2d %5d blk [%s]" % (B, best[0], best[0] / B, best[1], blocks, kinds))
    print("%-18s | %s" % (name, " | ".join(row)), flush=True)
