#!/usr/bin/env python3
"""Diagnostics: diff one tile config's static-mode outputs (limb planes) against config 0."""
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
cin, cout, k, s, h = 64, 256, 1, 1, 20
limbs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [27]
wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin + 5 * cout)
g = torch.Generator().manual_seed(11)
x = torch.relu(torch.randn(3, h, h, cin, generator=g)).to(gpu)
am = ops.act_absmax(x)
xq = ops.act_quantize(x, am, limbs)
rq = ops.act_quantize(torch.randn(3, h, h, cout, generator=g).clamp(-4, 4).to(gpu), torch.full((3,), 4.0, device=gpu), limbs)
shift = torch.linspace(-1, 1, cout, device=gpu)
for res in (False, True):
    kw = dict(residual_q=rq, residual_range=4.0) if res else {}
    outs = {}
    for c in [1] + cfgs:
        ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
        y, yq = ops.conv2d_q(xq, am, codes, offset, k, k, s, 0, step, shift, relu=True, tile_cfg=c,
                             emit_range=20.0, overflow=ovf, want_f32=True, **kw)
        outs[c] = (y.clone(), yq.clone())
    for c in cfgs:
        dy = (outs[c][0] != outs[1][0])
        dq = (outs[c][1] != outs[1][1])
        print("res", res, "cfg", c, "y diffs", int(dy.sum()), "yq diffs", int(dq.sum()), flush=True)
        if dq.any():
            idx = torch.nonzero(dq)[:6].tolist()
            print("   first yq diffs [l,n,h,w,c]:", idx)
            print("   pixel/channel hist:", torch.nonzero(dq)[:, 4].remainder(64).bincount(minlength=64)[:64].tolist()[:16])
