"""ResNet-18/34/50 with the reference's module tree and init, on QConv2d.

Mirrors resnet.py:22-265 of the reference so that (a) the search drivers can address
``net.layer{1..4}[b].conv{1,2,3}`` / ``.downsample`` exactly as before (resnet50_main.py:43,
189-197), (b) ``state_dict()`` keys are torchvision's (plus the qbits/qstep metadata buffers),
and (c) under the same ``torch.manual_seed`` the weights are bit-identical to the reference's
(same module construction order, same kaiming_normal_(fan_out, relu) pass, resnet.py:165-170;
checked against the golden checksums in tests/test_models.py).

``ResNet.forward`` runs ``smpq.engine.forward_fused`` (one fused HIP launch per quantized conv)
on GPU inputs in eval mode, and the plain module path otherwise.
"""
import torch
import torch.nn as nn

from . import engine
from .qconv import QConv2d

MODEL_URLS = {
    "resnet18": "https://download.pytorch.org/models/resnet18-5c106cde.pth",
    "resnet34": "https://download.pytorch.org/models/resnet34-333f7ec4.pth",
    "resnet50": "https://download.pytorch.org/models/resnet50-19c8e357.pth",
}


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    """3x3 conv, padding = dilation, no bias (resnet.py:22-25)."""
    return QConv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation,
                   groups=groups, bias=False, dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1):
    """1x1 conv, no bias (resnet.py:28-30)."""
    return QConv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    """Two 3x3 convs + identity (resnet.py:33-68)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        if groups != 1 or base_width != 64:
            raise ValueError("BasicBlock only supports groups=1 and base_width=64")
        if dilation > 1:
            raise NotImplementedError("Dilation > 1 not supported in BasicBlock")
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = norm_layer(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        shortcut = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        y += shortcut
        return self.relu(y)


class Bottleneck(nn.Module):
    """1x1 -> 3x3 (stride here: ResNet V1.5) -> 1x1 x4 (resnet.py:71-116)."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = norm_layer(width)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2 = norm_layer(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = norm_layer(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        shortcut = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        y += shortcut
        return self.relu(y)


class ResNet(nn.Module):
    """resnet.py:119-223. The stem and downsample convs are QConv2d too (never quantized by the
    drivers: they run with fp32 weights in 16-bit fixed point on the HIP kernel); fc stays fp32."""

    fused = True  # use smpq.engine on GPU in eval mode

    def __init__(self, block, layers, num_classes=1000, zero_init_residual=False, groups=1,
                 width_per_group=64, replace_stride_with_dilation=None, norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self._norm_layer = norm_layer
        self.block_name = block.__name__
        self.arch = layers
        self.inplanes = 64
        self.dilation = 1
        if replace_stride_with_dilation is None:
            replace_stride_with_dilation = [False, False, False]
        if len(replace_stride_with_dilation) != 3:
            raise ValueError("replace_stride_with_dilation should be None or a 3-element tuple, "
                             "got {}".format(replace_stride_with_dilation))
        self.groups = groups
        self.base_width = width_per_group
        self.conv1 = QConv2d(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = norm_layer(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2, dilate=replace_stride_with_dilation[0])
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2, dilate=replace_stride_with_dilation[1])
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2, dilate=replace_stride_with_dilation[2])
        self.layers = [self.layer1, self.layer2, self.layer3, self.layer4]
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        # same init pass, same module order as resnet.py:165-170 => same RNG stream
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        norm_layer = self._norm_layer
        previous_dilation = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       norm_layer(planes * block.expansion))
        mods = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width,
                      previous_dilation, norm_layer)]
        self.inplanes = planes * block.expansion
        mods += [block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                       dilation=self.dilation, norm_layer=norm_layer) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def _forward_impl(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            x = layer(x)
        return self.fc(torch.flatten(self.avgpool(x), 1))

    def forward(self, x):
        if self.fused and x.is_cuda and not self.training and self.dilation == 1 and self.groups == 1:
            return engine.forward_fused(self, x)
        return self._forward_impl(x)

    def _apply(self, fn, *args, **kwargs):
        # .to() / .cuda() / .half() that replace parameter or buffer tensors: drop the engine's cached
        # references (signature tensor list, captured graphs, ranges, fingerprints) so they are
        # rebuilt from the new tensors. A no-op .to() (the model already there: the reference's
        # evaluate_acc_loss_softmax calls net.to(device) on every evaluation, functions.py:97) keeps
        # them: dropping them would recalibrate, repack every weight and recapture every graph.
        def tensors():
            return [(id(t), t.data_ptr(), t.dtype, t.device) for t in self.parameters()] + \
                [(id(t), t.data_ptr(), t.dtype, t.device) for t in self.buffers()]
        before = tensors()
        out = super()._apply(fn, *args, **kwargs)
        if tensors() != before:
            for k in ("_smpq_graph", "_smpq_graphs", "_smpq_dyn", "_smpq_ranges", "_smpq_fp", "_smpq_pool"):
                self.__dict__.pop(k, None)
        return out


def _resnet(arch, block, layers, pretrained, progress, **kwargs):
    model = ResNet(block, layers, **kwargs)
    if pretrained:
        # resnet.py:228-231: a download; offline boxes can point SMPQ_PRETRAINED_DIR at local files
        import os
        local = os.environ.get("SMPQ_PRETRAINED_DIR")
        if local:
            path = os.path.join(local, os.path.basename(MODEL_URLS[arch]))
            state_dict = torch.load(path, map_location="cpu", weights_only=True)
        else:
            from torch.hub import load_state_dict_from_url
            state_dict = load_state_dict_from_url(MODEL_URLS[arch], progress=progress)
        model.load_state_dict(state_dict, strict=False)
    return model


def resnet18(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet18", BasicBlock, [2, 2, 2, 2], pretrained, progress, **kwargs)


def resnet34(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet34", BasicBlock, [3, 4, 6, 3], pretrained, progress, **kwargs)


def resnet50(pretrained=False, progress=True, **kwargs):
    return _resnet("resnet50", Bottleneck, [3, 4, 6, 3], pretrained, progress, **kwargs)
