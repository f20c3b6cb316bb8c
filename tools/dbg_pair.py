import sys, os
sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "semilayer-wise-mixed-precision-quantization_amd")); sys.path.insert(0, os.getcwd())
import torch
import __graft_entry__
__graft_entry__.build()
from test_gpu import build_model
from smpq import engine
gpu = torch.device("cuda")
net = build_model(gpu, "resnet50", "r50_mixed")
x = torch.randn(6, 3, 224, 224).to(gpu)
engine.USE_GRAPH[0] = False
with torch.no_grad():
    net(x); net(x)
for n, m in net.named_modules():
    if n.startswith("layer1") and hasattr(m, "last_path"):
        p = engine.conv_plan(m, None)
        print(n, m.last_path, None if p is None else (tuple(p[0].shape), p[1] is not None, p[4]))
