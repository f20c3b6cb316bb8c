"""ORACLE — test infrastructure only (see oracle/__init__.py).

The reference's CPU forward restated with the same torch CPU operators it runs (fp32
F.conv2d / batch_norm / relu / max_pool2d / adaptive_avg_pool2d / linear on oneDNN), over a
state dict. This is what ``net(x)`` at functions.py:113 executes on a CPU box (resnet.py:55-68,
97-116, 204-220), so it is used as ``bench.py``'s ``cpu_baseline`` ("port") and, being the
same operators in the same order, reproduces the reference's logits to the last bits
(tests/test_oracle_golden.py).
"""
import torch
import torch.nn.functional as F

from .forward_ref import ARCHS


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                        sd[p + ".bias"], False, 0.0, 1e-5)


@torch.no_grad()
def resnet_forward(arch, sd, x):
    kind, layers = ARCHS[arch]
    x = F.relu(_bn(F.conv2d(x, sd["conv1.weight"], None, 2, 3), sd, "bn1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, nblk in enumerate(layers):
        for b in range(nblk):
            stride = 2 if (li > 0 and b == 0) else 1
            p = "layer%d.%d" % (li + 1, b)
            identity = x
            if kind == "basic":
                out = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"], None, stride, 1), sd, p + ".bn1"))
                out = _bn(F.conv2d(out, sd[p + ".conv2.weight"], None, 1, 1), sd, p + ".bn2")
            else:
                out = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"], None, 1, 0), sd, p + ".bn1"))
                out = F.relu(_bn(F.conv2d(out, sd[p + ".conv2.weight"], None, stride, 1), sd, p + ".bn2"))
                out = _bn(F.conv2d(out, sd[p + ".conv3.weight"], None, 1, 0), sd, p + ".bn3")
            if (p + ".downsample.0.weight") in sd:
                identity = _bn(F.conv2d(x, sd[p + ".downsample.0.weight"], None, stride, 0), sd, p + ".downsample.1")
            out += identity
            x = F.relu(out)
    x = torch.flatten(F.adaptive_avg_pool2d(x, (1, 1)), 1)
    return F.linear(x, sd["fc.weight"], sd["fc.bias"])
