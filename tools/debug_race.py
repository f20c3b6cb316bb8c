#!/usr/bin/env python3
"""Diagnostics: repeat one static-mode conv per tile config and count runs whose outputs differ
from the register-staged reference config (a race shows up as intermittent mismatches)."""
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
from test_gpu import make_layer  # noqa: E402

gpu = torch.device("cuda")
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
cin, cout, k, s, h = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "64,256,1,1,20").split(","))
limbs = 3
cfgs = list(ops.tile_configs()) if sys.argv[1] == "all" else [int(c) for c in sys.argv[1].split(",")]
cfgs = [c for c in cfgs if ops._tile_fits(c, limbs, 1, False, cout, cin, k)]
wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin + 5 * cout)
g = torch.Generator().manual_seed(11)
x = torch.relu(torch.randn(3, h, h, cin, generator=g)).to(gpu)
am = ops.act_absmax(x)
xq = ops.act_quantize(x, am, limbs)
ho = (h + 2 * (k // 2) - k) // s + 1
rq = ops.act_quantize(torch.randn(3, ho, ho, cout, generator=g).clamp(-4, 4).to(gpu), torch.full((3,), 4.0, device=gpu), limbs)
shift = torch.linspace(-1, 1, cout, device=gpu)
ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=True, residual_q=rq, residual_range=4.0)
rng = float(ref.abs().max()) * 2.0
ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
variants = {"res+f32": dict(want_f32=True, residual_q=rq, residual_range=4.0)}
for name, kw in variants.items():
    y0, q0 = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=True, tile_cfg=1,
                          emit_range=rng, overflow=ovf, **kw)
    for c in cfgs:
        bad = 0
        for r in range(reps):
            y, q = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=True, tile_cfg=c,
                                emit_range=rng, overflow=ovf, **kw)
            if not torch.equal(q, q0) or not torch.equal(y, y0):
                bad += 1
                if bad == 1:
                    d = torch.nonzero(q != q0)
                    i0 = tuple(d[0].tolist())
                    print("  %s cfg %d rep %d: %d diffs, first %s, got %s want %s; pixels %s" % (
                        name, c, r, d.shape[0], i0, q[i0[:4]][i0[4] - (i0[4] % 16):][:16].tolist(),
                        q0[i0[:4]][i0[4] - (i0[4] % 16):][:16].tolist(),
                        sorted(set((x[1] * h * h + x[2] * h + x[3]) for x in d.tolist()))[:8]))
        if bad:
            print("%s cfg %d mismatching runs %d of %d" % (name, c, bad, reps), flush=True)
    print("checked configs", cfgs, flush=True)
