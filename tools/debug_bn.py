"""Debug: which side is stale after a BN buffer write through .data (test_cache_sees_every_kind_of_weight_change)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "semilayer-wise-mixed-precision-quantization_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import resnet  # noqa: E402
import functions  # noqa: E402,F401
from smpq import assignments, engine, stats  # noqa: E402
from smpq.qconv import QConv2d  # noqa: E402

gpu = torch.device("cuda:0")
mode = sys.argv[1] if len(sys.argv) > 1 else "dynamic"
what = sys.argv[2] if len(sys.argv) > 2 else "bn"
torch.manual_seed(0)
net = resnet.resnet50().to(gpu).eval()
assignments.apply_assignment(net, "r50_mixed", semantics="cpu")
x = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(31)).to(gpu)
engine.set_range_mode(mode)


def fresh_logits():
    fresh = resnet.resnet50().to(gpu).eval()
    fresh.load_state_dict(net.state_dict())
    for a, b in zip(net.modules(), fresh.modules()):
        if hasattr(a, "_bits_host"):
            b._bits_host = a._bits_host.copy()
            b._meta_gen += 1
    prev = engine.get_range_mode()
    engine.set_range_mode("dynamic")
    try:
        with torch.no_grad():
            return fresh(x)
    finally:
        engine.set_range_mode(prev)


def err(a, b):
    return ((a - b).abs().max() / b.abs().max()).item()


with torch.no_grad():
    net(x)
    y0 = net(x)
print("start", err(y0, fresh_logits()), dict(stats))
if what == "bn":
    bn = net.layer2[0].bn2
    bn.running_var.data.mul_(4.0)
else:
    import functions
    w = net.layer1[1].conv2.weight.data
    w[5] = functions.quantize_wgt(w[5].clone(), 4)
with torch.no_grad():
    y1 = net(x)
    print("first after write", err(y1, fresh_logits()), dict(stats))
    y2 = net(x)
    print("second", err(y2, fresh_logits()), dict(stats))
# drop every cache
for m in net.modules():
    for k in ("_fold_cache", "_s2d_cache"):
        if hasattr(m, k):
            delattr(m, k)
    if isinstance(m, QConv2d):
        m._content_gen += 1
for k in ("_smpq_graph", "_smpq_dyn", "_smpq_ranges"):
    if hasattr(net, k):
        setattr(net, k, None)
with torch.no_grad():
    y3 = net(x)
    y3 = net(x)
print("after cache drop", err(y3, fresh_logits()), "vs y2", err(y2, y3))
# the pure torch module path of the fresh model (no engine)
ref = fresh_logits()
print("fresh vs y0", err(ref, y0))
