import sys, numpy as np, torch
sys.path.insert(0, "semilayer-wise-mixed-precision-quantization_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from smpq import ops
import test_gpu as T
gpu = torch.device("cuda:0")
cin, cout, k, s, h = 64, 256, 1, 1, 20
limbs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
order = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [12, 19, 21, 13]
wd, step, codes, offset = T.make_layer(gpu, cin, cout, k, seed=cin + 7 * cout)
g = torch.Generator().manual_seed(12)
x = torch.relu(torch.randn(3, h, h, cin, generator=g)).to(gpu)
am = ops.act_absmax(x); xq = ops.act_quantize(x, am, limbs)
rq = ops.act_quantize(torch.randn(3, h, h, cout, generator=g).clamp(-4, 4).to(gpu), torch.full((3,), 4.0, device=gpu), limbs)
shift = torch.linspace(-1, 1, cout, device=gpu)
kw = dict(relu=True, residual_q=rq, residual_range=4.0)
ref = ops.conv2d_q(xq, am, codes, offset, k, k, s, 0, step, shift, **kw)
rng = float(ref.abs().max()) * 2.0
for rep in range(3):
    out = []
    for c in order:
        ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
        _, yq = ops.conv2d_q(xq, am, codes, offset, k, k, s, 0, step, shift, tile_cfg=c, emit_range=rng, overflow=ovf, want_f32=False, **kw)
        v = sum(yq[l].cpu().numpy().astype(np.int64) * 256 ** l for l in range(limbs))
        out.append((c, v))
    print("rep", rep, [(c, int((v != out[0][1]).sum())) for c, v in out])
# detail: first call of the order's first config vs cfg 12's planes
ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
planes = {}
for c in (order[0], 12):
    torch.manual_seed(5)
    _, yq = ops.conv2d_q(xq, am, codes, offset, k, k, s, 0, step, shift, tile_cfg=c, emit_range=rng, overflow=ovf, want_f32=False, **kw)
    planes[c] = yq.cpu().numpy().reshape(limbs, -1, cout)
a, b = planes[order[0]], planes[12]
for l in range(limbs):
    d = a[l] != b[l]
    rows, chans = np.nonzero(d)
    print("limb", l, "ndiff", d.sum(), "pixel rows mod 32:", np.unique(rows % 32)[:40], "chan mod 256 uniq:", np.unique(chans)[:20], "first rows", np.unique(rows)[:10])
