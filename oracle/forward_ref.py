"""ORACLE — test infrastructure only (see oracle/__init__.py).

float64 numpy restatement of the reference ResNet forward pass (eval mode), the
hot path named by BASELINE.json ``north_star``.

Reference:
  * ``resnet.py:22-30``   conv3x3 (pad 1) / conv1x1 (pad 0), bias=False
  * ``resnet.py:55-68``   BasicBlock.forward
  * ``resnet.py:97-116``  Bottleneck.forward (V1.5: stride on the 3x3)
  * ``resnet.py:181-202`` _make_layer (downsample = conv1x1(stride) + BN)
  * ``resnet.py:204-220`` ResNet._forward_impl (stem 7x7/s2/p3, BN, ReLU,
    maxpool 3x3/s2/p1, layer1..4, adaptive avgpool, flatten, fc)
BatchNorm in eval mode: ``(x - mean) / sqrt(var + eps) * gamma + beta``, eps = 1e-5.

The weights are whatever the caller passes (already fake-quantized the reference's
way by ``oracle.quant_ref``), so this restates exactly what ``net(x)`` computes at
``functions.py:113``.  It is slow and meant for batches of a few images.
"""
import numpy as np

ARCHS = {
    "resnet18": ("basic", [2, 2, 2, 2]),
    "resnet34": ("basic", [3, 4, 6, 3]),
    "resnet50": ("bottleneck", [3, 4, 6, 3]),
}


def conv2d(x, w, stride, pad):
    n, c, h, wd = x.shape
    co, ci, kh, kw = w.shape
    assert c == ci
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    ho = (h + 2 * pad - kh) // stride + 1
    wo = (wd + 2 * pad - kw) // stride + 1
    s = xp.strides
    cols = np.lib.stride_tricks.as_strided(
        xp, shape=(n, c, kh, kw, ho, wo),
        strides=(s[0], s[1], s[2], s[3], s[2] * stride, s[3] * stride))
    cols = cols.reshape(n, c * kh * kw, ho * wo)
    wm = w.reshape(co, -1).astype(np.float64)
    out = np.einsum("ok,nkp->nop", wm, cols, optimize=True)
    return out.reshape(n, co, ho, wo)


def batchnorm(x, sd, prefix, eps=1e-5):
    g = sd[prefix + ".weight"].astype(np.float64)
    b = sd[prefix + ".bias"].astype(np.float64)
    m = sd[prefix + ".running_mean"].astype(np.float64)
    v = sd[prefix + ".running_var"].astype(np.float64)
    inv = g / np.sqrt(v + eps)
    return (x - m[None, :, None, None]) * inv[None, :, None, None] + b[None, :, None, None]


def relu(x):
    return np.maximum(x, 0.0)


def maxpool3x3s2p1(x):
    n, c, h, w = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1), (1, 1)), constant_values=-np.inf)
    ho = (h + 2 - 3) // 2 + 1
    wo = (w + 2 - 3) // 2 + 1
    out = np.full((n, c, ho, wo), -np.inf)
    for i in range(3):
        for j in range(3):
            out = np.maximum(out, xp[:, :, i:i + 2 * ho:2, j:j + 2 * wo:2])
    return out


def block_forward(x, sd, p, kind, stride, has_ds):
    identity = x
    if kind == "basic":
        out = relu(batchnorm(conv2d(x, sd[p + ".conv1.weight"], stride, 1), sd, p + ".bn1"))
        out = batchnorm(conv2d(out, sd[p + ".conv2.weight"], 1, 1), sd, p + ".bn2")
    else:
        out = relu(batchnorm(conv2d(x, sd[p + ".conv1.weight"], 1, 0), sd, p + ".bn1"))
        out = relu(batchnorm(conv2d(out, sd[p + ".conv2.weight"], stride, 1), sd, p + ".bn2"))
        out = batchnorm(conv2d(out, sd[p + ".conv3.weight"], 1, 0), sd, p + ".bn3")
    if has_ds:
        identity = batchnorm(conv2d(x, sd[p + ".downsample.0.weight"], stride, 0), sd, p + ".downsample.1")
    return relu(out + identity)


def resnet_forward(arch, sd, x):
    """Full eval-mode forward; ``sd`` maps torchvision state_dict keys to numpy arrays."""
    kind, layers = ARCHS[arch]
    x = np.asarray(x, dtype=np.float64)
    x = relu(batchnorm(conv2d(x, sd["conv1.weight"], 2, 3), sd, "bn1"))
    x = maxpool3x3s2p1(x)
    for li, nblk in enumerate(layers):
        for b in range(nblk):
            stride = 2 if (li > 0 and b == 0) else 1
            p = "layer%d.%d" % (li + 1, b)
            has_ds = (p + ".downsample.0.weight") in sd
            x = block_forward(x, sd, p, kind, stride, has_ds)
    x = x.mean(axis=(2, 3))
    return x @ sd["fc.weight"].astype(np.float64).T + sd["fc.bias"].astype(np.float64)


def addressable_convs(arch):
    """The quantized ('addressable') convs in lnum order.

    R50: lnum = 3*(global block index) + {1,2,3} -> conv{1,2,3} (resnet50_main.py:81-136,189-197)
    R18/R34: lnum odd -> conv1, even -> conv2 (resnet18_main.py:86-115, 175-180), blocks in order.
    """
    kind, layers = ARCHS[arch]
    names = []
    for li, nblk in enumerate(layers):
        for b in range(nblk):
            p = "layer%d.%d" % (li + 1, b)
            convs = ["conv1", "conv2"] if kind == "basic" else ["conv1", "conv2", "conv3"]
            for c in convs:
                names.append(p + "." + c + ".weight")
    return names
