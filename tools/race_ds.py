#!/usr/bin/env python3
"""Diagnostics: repeat the first downsample conv of ResNet-50 (64 -> 256, 1x1, 56x56, fixed-point
weights with 3 limbs, static-range limb-plane output, no residual) per tile config and count runs
whose limb planes differ from the first run. Between runs, the output buffers of the previous run
are released and other garbage is written, so stale-memory reads show up too.
usage: python tools/race_ds.py [reps] [wlimbs] [batch]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"), REPO]
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from smpq import ops  # noqa: E402

gpu = torch.device("cuda")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
wl = int(sys.argv[2]) if len(sys.argv) > 2 else 3
B = int(sys.argv[3]) if len(sys.argv) > 3 else 6
cin, cout, h = 64, 256, 56
g = torch.Generator(device=gpu).manual_seed(0)
w = torch.randn(cout, cin, 1, 1, device=gpu, generator=g) * 0.1
step = None
if wl == 1:
    step = ops.quantize_channels_(w.reshape(cout, -1), [6] * cout)
codes, offset, wscale, st = ops.pack_weights_ex(w, step, wl)
x = torch.relu(torch.randn(B, h, h, cin, device=gpu, generator=g))
rng_in = float(x.abs().max()) * 2
am = torch.full((B,), rng_in, device=gpu)
xq = ops.act_quantize(x, am, 3)
shift = torch.linspace(-1, 1, cout, device=gpu)
ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
ref = ops.conv2d_q(xq, am, codes, offset if wl == 1 else None, 1, 1, 1, 0, wscale, shift)
rng = float(ref.abs().max()) * 2.0
for c in ops.tile_configs():
    if not ops._tile_fits(c, 3, wl, False, cout, cin, 1):
        continue
    base = None
    bad = 0
    for r in range(reps):
        junk = torch.randint(-128, 127, (3, B, h, h, cout), dtype=torch.int8, device=gpu)  # dirty the allocator
        del junk
        _, q = ops.conv2d_q(xq, am, codes, offset if wl == 1 else None, 1, 1, 1, 0, wscale, shift, relu=False,
                            tile_cfg=c, emit_range=rng, overflow=ovf, want_f32=False)
        if base is None:
            base = q.clone()
        elif not torch.equal(q, base):
            bad += 1
            if bad == 1:
                d = torch.nonzero(q != base)
                print("  cfg %d rep %d: %d diffs, first %s limbs %s" % (c, r, d.shape[0], d[0].tolist(),
                                                                      sorted(set(d[:, 0].tolist()))), flush=True)
    print("cfg %d kind %d tile %s: %d of %d runs differ" % (c, ops.tile_kind(c), ops.tile_configs()[c], bad, reps - 1),
          flush=True)
