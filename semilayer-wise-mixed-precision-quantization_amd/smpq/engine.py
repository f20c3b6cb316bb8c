"""Fused eval-mode ResNet forward on the HIP path (NHWC end to end).

Restates ``ResNet._forward_impl`` (resnet.py:204-220), ``BasicBlock.forward`` (resnet.py:55-68)
and ``Bottleneck.forward`` (resnet.py:97-116) with every quantized conv + its BatchNorm
(+ residual add) (+ ReLU) as ONE ``smpq_conv2d_fwd`` launch:

  * activations stay NHWC fp32 in HBM between layers (no layout round trips);
  * each conv epilogue also produces the per-image max|y| that the NEXT conv's activation
    quantizer needs (atomicMax), so there is no separate range pass;
  * BN (eval) is folded per output channel: a = gamma / sqrt(var + eps), b = beta - mean * a,
    and the weight step is folded into the same column scale.

Unquantized parts stay fp32 exactly like the reference: the 7x7 stem + BN + ReLU + maxpool,
the downsample 1x1 conv + BN (resnet.py:188-192), avgpool and fc run as torch/MIOpen ops on
channels_last tensors, as does any conv that is not fully quantized (see qconv.py).
"""
import torch
import torch.nn.functional as F

from . import ops
from .qconv import QConv2d, stats


def _bn_fold(bn):
    inv = torch.rsqrt(bn.running_var.float() + bn.eps)
    a = bn.weight.float() * inv if bn.affine else inv
    b = (bn.bias.float() if bn.affine else torch.zeros_like(a)) - bn.running_mean.float() * a
    return a, b


def _bn_key(bn):
    ts = [bn.running_mean, bn.running_var]
    if bn.affine:
        ts += [bn.weight, bn.bias]
    return tuple((t.data_ptr(), t._version) for t in ts) + (bn.eps,)


def conv_plan(conv, bn):
    """(codes, offset, col_scale, col_shift) for the fused kernel, or None (fp32 path)."""
    if not isinstance(conv, QConv2d):
        return None
    if conv.stride[0] != conv.stride[1] or conv.padding[0] != conv.padding[1] or conv.bias is not None:
        return None
    pk = conv.packed()
    if pk is None:
        return None
    key = (conv._pack_key(), _bn_key(bn))
    cache = getattr(conv, "_fold_cache", None)
    if cache is not None and cache[0] == key:
        return cache[1]
    with torch.no_grad():
        a, b = _bn_fold(bn)
        col_scale = (conv.qstep.float() * a).contiguous()
        col_shift = b.contiguous()
    plan = (pk[0], pk[1], col_scale, col_shift)
    conv._fold_cache = (key, plan)
    return plan


def _to_nchw(x_nhwc):
    return x_nhwc.permute(0, 3, 1, 2)


def _to_nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def conv_bn_act(conv, bn, x, x_amax, relu, residual=None, y_amax=None):
    """y = act(bn(conv(x)) [+ residual]) on NHWC fp32; fills y_amax (per image max|y|) if given."""
    plan = conv_plan(conv, bn)
    if plan is not None:
        codes, offset, col_scale, col_shift = plan
        stats["hip_conv"] += 1
        conv.last_path = "hip"
        return ops.conv2d_nhwc(x, x_amax, codes, offset, conv.kernel_size[0], conv.kernel_size[1],
                               conv.stride[0], conv.padding[0], col_scale, col_shift,
                               residual=residual, relu=relu, y_absmax=y_amax)
    # fp32 path (unquantized weights: the reference's own arithmetic, on MIOpen)
    stats["fp32_conv"] += 1
    conv.last_path = "fp32"
    y = F.conv2d(_to_nchw(x), conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation, conv.groups)
    y = F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
    if residual is not None:
        y = y + _to_nchw(residual)
    if relu:
        y = F.relu(y)
    y = _to_nhwc(y)
    if y_amax is not None:
        ops.act_absmax(y, out=y_amax)
    return y


def _downsample(ds, x):
    conv, bn = ds[0], ds[1]
    plan = conv_plan(conv, bn)
    if plan is not None:
        amax = ops.act_absmax(x)
        return conv_bn_act(conv, bn, x, amax, relu=False)
    y = F.conv2d(_to_nchw(x), conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation, conv.groups)
    y = F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
    return _to_nhwc(y)


def block_forward(blk, x, x_amax, amax_bank, idx):
    """One BasicBlock / Bottleneck on NHWC x. Returns (out, out_amax, next bank index)."""
    identity = x
    if blk.downsample is not None:
        identity = _downsample(blk.downsample, x)
    if hasattr(blk, "conv3"):  # Bottleneck (resnet.py:97-116)
        t1 = conv_bn_act(blk.conv1, blk.bn1, x, x_amax, True, y_amax=amax_bank[idx])
        t2 = conv_bn_act(blk.conv2, blk.bn2, t1, amax_bank[idx], True, y_amax=amax_bank[idx + 1])
        out = conv_bn_act(blk.conv3, blk.bn3, t2, amax_bank[idx + 1], True, residual=identity,
                          y_amax=amax_bank[idx + 2])
        return out, amax_bank[idx + 2], idx + 3
    # BasicBlock (resnet.py:55-68)
    t1 = conv_bn_act(blk.conv1, blk.bn1, x, x_amax, True, y_amax=amax_bank[idx])
    out = conv_bn_act(blk.conv2, blk.bn2, t1, amax_bank[idx], True, residual=identity,
                      y_amax=amax_bank[idx + 1])
    return out, amax_bank[idx + 1], idx + 2


def forward_fused(model, x):
    """Eval-mode forward of an smpq ResNet on the GPU; returns logits [n, num_classes]."""
    x = x.float().contiguous(memory_format=torch.channels_last)
    h = model.conv1(x)
    h = model.bn1(h)
    h = model.relu(h)
    h = model.maxpool(h)
    h = _to_nhwc(h)
    blocks = [b for layer in (model.layer1, model.layer2, model.layer3, model.layer4) for b in layer]
    nconv = sum(3 if hasattr(b, "conv3") else 2 for b in blocks)
    amax_bank = torch.zeros(nconv + 1, h.shape[0], dtype=torch.float32, device=h.device)
    ops.act_absmax(h, out=amax_bank[nconv])
    amax = amax_bank[nconv]
    idx = 0
    for blk in blocks:
        h, amax, idx = block_forward(blk, h, amax, amax_bank, idx)
    feat = h.mean(dim=(1, 2))
    return model.fc(feat)
