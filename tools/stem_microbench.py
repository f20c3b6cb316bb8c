"""Time the fused stem (conv1 + bn1 + relu + maxpool, ops.stem_pool_s2d) against the two-launch
path (tuned stem_conv_s2d + maxpool_limbs) on ResNet-50's stem shape.
usage: python tools/stem_microbench.py [batch] [limbs] [reps]   (SMPQ_LIB selects an ablation build)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "semilayer-wise-mixed-precision-quantization_amd"))
from smpq import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
limbs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
gpu = torch.device("cuda:0")
g = torch.Generator().manual_seed(1)
wt = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(gpu)
x = torch.randn(n, 3, 224, 224, generator=g).to(gpu)
am = ops.act_absmax(x)
codes, wscale = ops.pack_weights_s2d(wt, max(2, limbs))
cs = (wscale * torch.linspace(0.5, 2, 64, device=gpu)).contiguous()
sh = torch.linspace(-1, 1, 64, device=gpu).contiguous()
xs = ops.image_quantize_s2d(x, am, limbs)
ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
rng = 50.0


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


fused = timed(lambda: ops.stem_pool_s2d(xs, am, codes, 224, 224, cs, sh, emit_range=rng, overflow=ovf))
if os.environ.get("STAMPS"):  # a -DSMPQ_SP_DIAG=8 build: phase timestamps of workgroup 0
    yq = ops.stem_pool_s2d(xs, am, codes, 224, 224, cs, sh, emit_range=rng, overflow=ovf)
    torch.cuda.synchronize()
    d = yq.reshape(-1)[:8 * 16 * 8 * 16].view(torch.int64).reshape(8, 16, 8, 2).cpu()
    t0 = d[:, 0, 0, 0].min()
    r0 = d[:, 0, 0, 1].min()
    clk = (d[:, :, 7, 0].max() - t0).item() / ((d[:, :, 7, 1].max() - r0).item() / 100e6) / 1e9
    print("clock ~%.2f GHz; per wave, per step: cycles of [h0 dma, h0 work, h0 wait, h0 barrier, h1 work, h1 wait, "
          "h1 barrier]" % clk)
    for w in (0, 4):
        for k in range(2, 8):
            e = d[w, k, :, 0].tolist()
            if w == 0:
                e[1] = e[0]
            nxt = d[w, k + 1, 0, 0].item()
            seg = [e[1] - e[0], e[2] - e[1], e[3] - e[2], e[4] - e[3], e[6] - e[4], e[7] - e[6], nxt - e[7]]
            print("wave %d step %d: %s total %d" % (w, k, seg, nxt - e[0]))
if os.environ.get("SMPQ_LIB"):
    print("fused stem+pool n=%d L=%d: %.1f us (%s)" % (n, limbs, fused, os.environ["SMPQ_LIB"]))
    sys.exit(0)


def two():
    _, yq = ops.tuned_stem_conv_s2d(xs, am, codes, 224, 224, cs, sh, relu=True, emit_range=rng, overflow=ovf,
                                    want_f32=False)
    return ops.maxpool_limbs(yq)


two_t = timed(two)
same = torch.equal(two(), ops.stem_pool_s2d(xs, am, codes, 224, 224, cs, sh, emit_range=rng, overflow=ovf))
print("fused stem+pool n=%d L=%d: %.1f us; stem conv + maxpool_limbs: %.1f us; bitwise equal: %s"
      % (n, limbs, fused, two_t, same))
