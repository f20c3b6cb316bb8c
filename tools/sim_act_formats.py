"""Round 3: logit error of other activation formats on the golden parity models (CPU, float64
restatement of the forward, each conv input rounded as the format would; unquantized weights
optionally rounded too). fp16 / bf16 activations vs the reference CPU logits. Diagnostics only:
    python tools/sim_act_formats.py"""
import sys, numpy as np, torch, torch.nn.functional as F
sys.path.insert(0, "/root/repo/semilayer-wise-mixed-precision-quantization_amd"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo")
import test_gpu as T
from oracle.forward_ref import ARCHS
torch.set_num_threads(8)
g = T._golden()
def fwd(arch, sd, x, ract, rw_unq, qset):
    kind, layers = ARCHS[arch]
    def conv(x, name, s, p):
        w = sd[name].double()
        if name not in qset: w = rw_unq(w)
        return F.conv2d(ract(x), w, None, s, p)
    def bn(x, p):
        return F.batch_norm(x, sd[p + ".running_mean"].double(), sd[p + ".running_var"].double(), sd[p + ".weight"].double(), sd[p + ".bias"].double(), False, 0.0, 1e-5)
    x = F.relu(bn(conv(x, "conv1.weight", 2, 3), "bn1")); x = F.max_pool2d(x, 3, 2, 1)
    for li, nblk in enumerate(layers):
        for b in range(nblk):
            stride = 2 if (li > 0 and b == 0) else 1
            p = "layer%d.%d" % (li + 1, b); identity = x
            if kind == "basic":
                out = F.relu(bn(conv(x, p+".conv1.weight", stride, 1), p+".bn1")); out = bn(conv(out, p+".conv2.weight", 1, 1), p+".bn2")
            else:
                out = F.relu(bn(conv(x, p+".conv1.weight", 1, 0), p+".bn1")); out = F.relu(bn(conv(out, p+".conv2.weight", stride, 1), p+".bn2")); out = bn(conv(out, p+".conv3.weight", 1, 0), p+".bn3")
            if (p + ".downsample.0.weight") in sd:
                identity = bn(conv(x, p+".downsample.0.weight", stride, 0), p+".downsample.1")
            x = F.relu(out + identity)
    x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
    return F.linear(x, sd["fc.weight"].double(), sd["fc.bias"].double())
ident = lambda t: t
f16 = lambda t: t.half().double()
bf16 = lambda t: t.bfloat16().double()
def f16x2(t):
    hi = t.half().double(); return hi + (t - hi).half().double()
for case, arch, assign, batch in [("r18_u8_cal","resnet18","r18_u8",16),("r50_mixed_cal","resnet50","r50_mixed",8),("r34_4bit_cal","resnet34","r34_4bit",8),("r50_mixed","resnet50","r50_mixed",2)]:
    net = T.build_model(torch.device("cpu"), arch, assign, case if case.endswith("_cal") else None)
    sd = net.state_dict()
    qset = {n for n, m in net.named_modules() if getattr(m, "qbits", None) is not None}
    qset = {n + ".weight" for n in qset}
    x = torch.randn(batch, 3, 224, 224, generator=torch.Generator().manual_seed(1)).double()
    ref = g[case + "/logits"].astype(np.float64)
    srt = np.sort(ref, 1); print(case, "nq", len(qset), "min margin %.2e" % ((srt[:, -1] - srt[:, -2]).min() / np.abs(ref).max()))
    for nm, ra, rw in [("exact", ident, ident), ("act f16, unq w exact", f16, ident), ("act f16, unq w f16", f16, f16), ("act f16, unq w f16x2", f16, f16x2), ("act bf16", bf16, ident)]:
        with torch.no_grad(): y = fwd(arch, sd, x, ra, rw, qset).numpy()
        rel = np.abs(y - ref).max() / np.abs(ref).max()
        per = (np.abs(y - ref).max(1) / np.abs(ref).max(1)).max()
        print("  %-24s rel %.2e  per-image %.2e  top1 %d/%d" % (nm, rel, per, (y.argmax(1) == ref.argmax(1)).sum(), batch))
