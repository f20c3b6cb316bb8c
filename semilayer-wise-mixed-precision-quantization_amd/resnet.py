"""Drop-in for the reference's ``resnet`` module (resnet.py:1-265).

``import resnet`` from this directory gives the same names — ``ResNet``, ``resnet18``,
``resnet34``, ``resnet50``, ``conv3x3``, ``conv1x1``, ``BasicBlock``, ``Bottleneck``,
``model_urls`` — backed by smpq's QConv2d and the fused HIP forward.
"""
from smpq.models import (BasicBlock, Bottleneck, MODEL_URLS, ResNet, conv1x1, conv3x3,  # noqa: F401
                         resnet18, resnet34, resnet50)

model_urls = MODEL_URLS
__all__ = ["ResNet", "resnet18", "resnet34", "resnet50"]
