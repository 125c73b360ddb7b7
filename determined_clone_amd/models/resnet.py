"""ResNet-50 (v1.5) for the headline benchmark trial.

The reference benchmarks torchvision's ``resnet50`` inside a PyTorchTrial
(`examples/deepspeed_autotune/torchvision/`); torchvision is not part of this image, so the
architecture is defined here. It is laid out for MI355X rather than copied:

* activations are NHWC (``channels_last``) bf16 end to end, so MIOpen picks its NHWC
  implicit-GEMM (MFMA) convolutions and no layout transposes run between layers;
* every ``BatchNorm -> (+ residual) -> ReLU`` tail is ONE module, ``BatchNormAct2d``, which on a
  GPU runs the hand-written NHWC HIP kernels in ``ops/csrc/batchnorm.hip`` (stats + apply + add +
  ReLU in two passes over HBM instead of four separate PyTorch ops); BN affine params and running
  stats stay fp32 while activations are bf16;
* 3x3 convolutions run on the hand-written implicit-GEMM MFMA kernel (``ops/csrc/conv_igemm.hip``,
  forward + stride-1 data gradient), whose forward epilogue also reduces the following
  BatchNorm's statistics;
* 1x1 convolutions go through ``ops.conv.pointwise_conv``: per shape and direction the fastest of
  MIOpen, hipBLASLt and the implicit GEMM (whose forward epilogue also reduces the next
  BatchNorm's statistics);
* a downsampling block's tail ``relu(bn3(conv3(..)) + bn_ds(proj(x)))`` is ONE fused op
  (``ops.batchnorm.batch_norm_act_dual``): the projection shortcut's BatchNorm is applied inside
  bn3's apply pass (its output is never written) and both BatchNorms' backward share one
  statistics pass and one apply pass (``DCA_BN_DUAL=0`` keeps two separate BatchNorms);
* the classifier is a plain PyTorch op (<2 % of step time).
"""
import os
from typing import List, Optional, Type

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_clone_amd.ops import batchnorm as bn_ops
from determined_clone_amd.ops import conv as conv_ops
from determined_clone_amd.ops.conv import pointwise_conv, pointwise_dual

BN_DUAL = os.environ.get("DCA_BN_DUAL", "1") != "0"


class BatchNormAct2d(nn.BatchNorm2d):
    """BatchNorm2d with an optional fused residual add and ReLU.

    ``forward(x, residual=None)`` computes ``act(bn(x) + residual)``. Parameters/buffers have the
    same names as ``nn.BatchNorm2d`` so state dicts interchange with torchvision checkpoints.
    """

    def __init__(self, num_features: int, relu: bool = True, eps: float = 1e-5,
                 momentum: float = 0.1) -> None:
        super().__init__(num_features, eps=eps, momentum=momentum)
        self.relu = relu

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                fuse_residual_grad: bool = False) -> torch.Tensor:
        return bn_ops.batch_norm_act(
            x,
            self.weight,
            self.bias,
            self.running_mean,
            self.running_var,
            residual=residual,
            training=self.training,
            momentum=self.momentum,
            eps=self.eps,
            relu=self.relu,
            num_batches_tracked=self.num_batches_tracked,
            fuse_residual_grad=fuse_residual_grad,
        )


def _conv(cin: int, cout: int, k: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=k, stride=stride, padding=k // 2, bias=False)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1) -> None:
        super().__init__()
        cout = width * self.expansion
        self.conv1 = _conv(cin, width, 1)
        self.bn1 = BatchNormAct2d(width)
        self.conv2 = _conv(width, width, 3, stride)  # v1.5: stride on the 3x3
        self.bn2 = BatchNormAct2d(width)
        self.conv3 = _conv(width, cout, 1)
        self.bn3 = BatchNormAct2d(cout)  # bn3 + residual + relu fused
        self.downsample: Optional[nn.Module] = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(
                _conv(cin, cout, 1, stride), BatchNormAct2d(cout, relu=False)
            )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # 1x1/stride-1 convolutions: ops/conv.py (MIOpen, or opt-in MFMA kernels whose forward
        # epilogue also reduces the following BatchNorm's statistics)
        if self.downsample is None:
            identity = x
            out = self.bn1(pointwise_conv(self.conv1, x, self.bn1.training))
        else:
            # conv1 and the projection shortcut read the same x: one op, one input gradient
            # (the shortcut's strided backward-data is accumulated in place, ops/conv.py)
            ds_conv, ds_bn = self.downsample
            y1, yd = pointwise_dual(self.conv1, ds_conv, x, self.bn1.training)
            out = self.bn1(y1)
            if BN_DUAL and self.bn3.relu and not ds_bn.relu:
                out = self.bn2(conv_ops.spatial_conv(self.conv2, out, self.bn2.training))
                # relu(bn3(conv3) + bn_ds(proj)): one fused op, the shortcut BN never written
                return bn_ops.batch_norm_act_dual(pointwise_conv(self.conv3, out, self.bn3.training),
                                                  self.bn3, yd, ds_bn)
            identity = ds_bn(yd)
        # 3x3: implicit-GEMM MFMA kernel whose epilogue also reduces bn2's statistics
        out = self.bn2(conv_ops.spatial_conv(self.conv2, out, self.bn2.training))
        # identity shortcut: x also feeds conv1, so its gradient can be summed inside the
        # producer's BN backward (no separate autograd add)
        return self.bn3(pointwise_conv(self.conv3, out, self.bn3.training), residual=identity,
                        fuse_residual_grad=self.downsample is None)


class ResNet(nn.Module):
    def __init__(self, layers: List[int], num_classes: int = 1000,
                 block: Type[Bottleneck] = Bottleneck, zero_init_residual: bool = True) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNormAct2d(64)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        cin = 64
        stages = []
        for i, (n, width) in enumerate(zip(layers, [64, 128, 256, 512])):
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(block(cin, width, stride))
                cin = width * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.fc = nn.Linear(cin, num_classes)

        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # stem: conv -> fused BN + ReLU + 3x3/2 max-pool (the 112x112 pre-pool activation is never
        # written; its gradient is gathered inside the BN backward)
        bn = self.bn1
        # (the stem kernel reduces the BatchNorm's batch statistics in its epilogue)
        x = conv_ops.stem_conv(self.conv1, x, bn_stats=bn.training)
        x = bn_ops.batch_norm_relu_maxpool(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, training=bn.training,
                                           momentum=bn.momentum, eps=bn.eps,
                                           num_batches_tracked=bn.num_batches_tracked)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = bn_ops.global_avg_pool(x)
        return self.fc(x)


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet([3, 4, 6, 3], num_classes=num_classes)


def resnet18_bottleneck_tiny(num_classes: int = 10) -> ResNet:
    """A 4-block bottleneck ResNet for fast CPU tests of the same code path."""
    return ResNet([1, 1, 1, 1], num_classes=num_classes)


def to_mi355x_layout(model: nn.Module, dtype: torch.dtype = torch.bfloat16) -> nn.Module:
    """Convert a ResNet to the MI355X training layout: NHWC, conv/fc weights in ``dtype``,
    BatchNorm affine params and running stats kept in fp32 (the fused BN kernels read them as
    fp32)."""
    model = model.to(memory_format=torch.channels_last)
    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            m.to(dtype)
    return model
