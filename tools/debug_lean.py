import sys, numpy as np, torch
sys.path.insert(0, "semilayer-wise-mixed-precision-quantization_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from smpq import ops
import test_gpu as T
gpu = torch.device("cuda:0")
for (cin, cout, k, s, h) in [(64, 256, 1, 1, 20), (256, 256, 1, 1, 12)]:
  for limbs in (2, 3):
    for use_res in (True, False):
      for relu in (True, False):
        wd, step, codes, offset = T.make_layer(gpu, cin, cout, k, seed=cin + 7 * cout)
        g = torch.Generator().manual_seed(12)
        x = torch.relu(torch.randn(3, h, h, cin, generator=g)).to(gpu)
        am = ops.act_absmax(x); xq = ops.act_quantize(x, am, limbs)
        ho = h
        rq = ops.act_quantize(torch.randn(3, ho, ho, cout, generator=g).clamp(-4, 4).to(gpu), torch.full((3,), 4.0, device=gpu), limbs)
        shift = torch.linspace(-1, 1, cout, device=gpu)
        kw = dict(relu=relu, residual_q=rq if use_res else None, residual_range=4.0 if use_res else None)
        ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, 0, step, shift, **kw)
        rng = float(ref.abs().max()) * 2.0
        res = {}
        bad = []
        for c in ops.tile_configs():
            if not ops._tile_fits(c, limbs, 1, False, cout, cin, k) or ops.tile_kind(c) < 2: continue
            ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
            _, yq = ops.conv2d_q(xq, am, codes, offset, k, k, s, 0, step, shift, tile_cfg=c, emit_range=rng, overflow=ovf, want_f32=False, **kw)
            res[c] = sum(yq[l].cpu().numpy().astype(np.int64) * 256 ** l for l in range(limbs))
            _, yqf = ops.conv2d_q(xq, am, codes, offset, k, k, s, 0, step, shift, tile_cfg=c, emit_range=rng, overflow=ovf, want_f32=True, **kw)
            full = sum(yqf[l].cpu().numpy().astype(np.int64) * 256 ** l for l in range(limbs))
            d = res[c] - full
            if np.abs(d).max() > 1: bad.append((c, int((np.abs(d) > 1).sum())))
        print((cin, cout, h), "L", limbs, "res", use_res, "relu", relu, "bad cfgs:", bad)
