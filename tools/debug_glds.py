#!/usr/bin/env python3
"""Diagnostics: diff an LDS-DMA tile config against the register-staged reference config."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from smpq import ops  # noqa: E402
from test_gpu import make_layer  # noqa: E402

gpu = torch.device("cuda")
cin, cout, k, s, h, limbs = 64, 256, 1, 1, 20, int(sys.argv[1]) if len(sys.argv) > 1 else 1
wd, step, codes, offset = make_layer(gpu, cin, cout, k, seed=cin + 5 * cout)
g = torch.Generator().manual_seed(11)
x = torch.relu(torch.randn(3, h, h, cin, generator=g)).to(gpu)
am = ops.act_absmax(x)
xq = ops.act_quantize(x, am, limbs)
ho = h
resf = torch.randn(3, ho, ho, cout, generator=g).clamp(-4, 4).to(gpu)
rq = ops.act_quantize(resf, torch.full((3,), 4.0, device=gpu), limbs)
shift = torch.linspace(-1, 1, cout, device=gpu)
for cfg in (12, 15):
    for name, kw in [("noresid", {}), ("resq", dict(residual_q=rq, residual_range=4.0)),
                     ("resf", dict(residual=resf))]:
        a = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=False, tile_cfg=0, **kw)
        b = ops.conv2d_q(xq, am, codes, offset, k, k, s, k // 2, step, shift, relu=False, tile_cfg=cfg, **kw)
        d = (a - b).abs()
        nz = torch.nonzero(d > 0)
        print(cfg, name, "maxdiff %.3e" % d.max().item(), "ndiff", nz.shape[0], "of", d.numel(), flush=True)
        if nz.shape[0]:
            idx = nz[:8].tolist()
            for i in idx:
                print("   ", i, a[tuple(i)].item(), b[tuple(i)].item())
            ch = nz[:, 3].cpu().numpy()
            print("    channel mod 16 hist", np.bincount(ch % 16, minlength=16).tolist())
            px = (nz[:, 1] * ho + nz[:, 2]).cpu().numpy()
            print("    pixel mod 16 hist", np.bincount(px % 16, minlength=16).tolist())
