"""Round 3: per-tensor sensitivity of the R50 parity model to 16-bit (vs 24-bit) fixed-point
activation codes with static per-layer ranges (max over the batch x 2, as engine.py): one tensor at
16 bits at a time, then the deep tail of the network at 16 bits. CPU float64 restatement; numbers in
DESIGN.md 4c. Diagnostics only:  python tools/sim_limb_sensitivity.py"""
import sys, numpy as np, torch, torch.nn.functional as F
sys.path.insert(0, "/root/repo/semilayer-wise-mixed-precision-quantization_amd"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo")
import test_gpu as T
from oracle.forward_ref import ARCHS
torch.set_num_threads(8)
g = T._golden()
def fwd(arch, sd, x, bits_of, ranges=None, rec=None):
    kind, layers = ARCHS[arch]
    idx = [0]
    def q(t):
        i = idx[0]; idx[0] += 1
        if rec is not None: rec.append(t.abs().max().item())
        b = bits_of(i)
        if b is None or ranges is None: return t
        Q = 2.0 ** (b - 1) - 1; r = ranges[i] * 2.0
        return torch.round(t / r * Q) * r / Q
    def conv(x, name, s, p):
        return F.conv2d(x, sd[name].double(), None, s, p)
    def bn(x, p):
        return F.batch_norm(x, sd[p + ".running_mean"].double(), sd[p + ".running_var"].double(), sd[p + ".weight"].double(), sd[p + ".bias"].double(), False, 0.0, 1e-5)
    x = F.relu(bn(conv(x, "conv1.weight", 2, 3), "bn1")); x = F.max_pool2d(x, 3, 2, 1)
    x = q(x)
    for li, nblk in enumerate(layers):
        for b in range(nblk):
            stride = 2 if (li > 0 and b == 0) else 1
            p = "layer%d.%d" % (li + 1, b); identity = x
            out = q(F.relu(bn(conv(x, p+".conv1.weight", 1, 0), p+".bn1")))
            out = q(F.relu(bn(conv(out, p+".conv2.weight", stride, 1), p+".bn2")))
            out = bn(conv(out, p+".conv3.weight", 1, 0), p+".bn3")
            if (p + ".downsample.0.weight") in sd:
                identity = q(bn(conv(x, p+".downsample.0.weight", stride, 0), p+".downsample.1"))
            x = q(F.relu(out + identity))
    x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
    return F.linear(x, sd["fc.weight"].double(), sd["fc.bias"].double())
case, arch, assign, batch = "r50_mixed_cal", "resnet50", "r50_mixed", 8
net = T.build_model(torch.device("cpu"), arch, assign, case)
sd = net.state_dict()
x = torch.randn(batch, 3, 224, 224, generator=torch.Generator().manual_seed(1)).double()
ref = g[case + "/logits"].astype(np.float64)
rec = []
with torch.no_grad(): y0 = fwd(arch, sd, x, lambda i: None, None, rec).numpy()
ranges = rec; n = len(ranges)
def err(bits_of):
    with torch.no_grad(): y = fwd(arch, sd, x, bits_of, ranges).numpy()
    return np.abs(y - ref).max() / np.abs(ref).max(), (y.argmax(1) == ref.argmax(1)).sum()
print("tensors", n, "exact %.2e" % (np.abs(y0 - ref).max() / np.abs(ref).max()))
print("all 24: %.2e %d" % err(lambda i: 24))
print("all 16: %.2e %d" % err(lambda i: 16))
print("all 20: %.2e %d" % err(lambda i: 20))
res = []
for j in range(n) if "--per-tensor" in sys.argv else []:
    e, t = err(lambda i: 16 if i == j else 24)
    res.append(e); print("tensor %2d at 16b: %.2e top1 %d" % (j, e, t), flush=True)
for j0 in (24, 28, 31, 34, 37, 40, 43, 46):
    print("tensors >= %d at 16b: %.2e top1 %d" % ((j0,) + err(lambda i: 16 if i >= j0 else 24)), flush=True)
print("layer4 only 3x3 inputs+conv1 out 16b: %.2e %d" % err(lambda i: 16 if i in (43,44,47,48,50,51) else 24))
