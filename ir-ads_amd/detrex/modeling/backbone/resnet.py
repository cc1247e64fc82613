"""ResNet-50 with frozen BatchNorm, as the vCLR DINO config builds it (dino_r50.py:23-32:
detectron2 ResNet, BasicStem, make_default_stages(depth=50, stride_in_1x1=False, norm="FrozenBN"),
out_features res3 / res4 / res5, freeze_at=1; the reference's own copy of that design is
detrex/modeling/backbone/resnet.py:117-625).  Same module tree and state-dict keys
(``stem.conv1.weight``, ``res2.0.conv1.norm.running_mean``, ``res3.0.shortcut.weight`` ...), so a
detectron2 R50 checkpoint loads unchanged.  Plain PyTorch convolutions (MIOpen): the backbone
feeds the MSDA hot path, it is not part of it."""
import torch
import torch.nn as nn
import torch.nn.functional as F


class FrozenBatchNorm2d(nn.Module):
    """BatchNorm with fixed statistics and affine parameters (buffers, never trained):
    y = x · weight / sqrt(running_var + eps) + (bias − running_mean · that scale)."""

    def __init__(self, num_features, eps=1e-5):
        super().__init__()
        self.num_features, self.eps = num_features, eps
        self.register_buffer("weight", torch.ones(num_features))
        self.register_buffer("bias", torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features) - eps)

    def forward(self, x):
        scale = self.weight * (self.running_var + self.eps).rsqrt()
        bias = self.bias - self.running_mean * scale
        return x * scale.view(1, -1, 1, 1).to(x.dtype) + bias.view(1, -1, 1, 1).to(x.dtype)


class _ConvNorm(nn.Conv2d):
    """detectron2's Conv2d(norm=...): convolution then the norm (``<name>.norm.*`` keys)."""

    def __init__(self, *args, norm=None, **kwargs):
        super().__init__(*args, **kwargs)
        self.norm = norm

    def forward(self, x):
        x = super().forward(x)
        return self.norm(x) if self.norm is not None else x


def _norm(norm, channels):
    if norm == "FrozenBN":
        return FrozenBatchNorm2d(channels)
    if norm == "BN":
        return nn.BatchNorm2d(channels)
    if norm in (None, ""):
        return None
    raise ValueError(f"unsupported norm {norm!r}")


class BasicStem(nn.Module):
    """7x7 stride-2 convolution + norm + ReLU + 3x3 stride-2 max-pool (stride 4)."""

    def __init__(self, in_channels=3, out_channels=64, norm="BN"):
        super().__init__()
        self.in_channels, self.out_channels, self.stride = in_channels, out_channels, 4
        self.conv1 = _ConvNorm(in_channels, out_channels, kernel_size=7, stride=2, padding=3, bias=False,
                               norm=_norm(norm, out_channels))

    def forward(self, x):
        return F.max_pool2d(F.relu_(self.conv1(x)), kernel_size=3, stride=2, padding=1)


class BottleneckBlock(nn.Module):
    """1x1 -> 3x3 (stride here: stride_in_1x1=False) -> 1x1, projection shortcut when the width changes."""

    def __init__(self, in_channels, out_channels, *, bottleneck_channels, stride=1, norm="BN", stride_in_1x1=False):
        super().__init__()
        self.in_channels, self.out_channels, self.stride = in_channels, out_channels, stride
        self.shortcut = (_ConvNorm(in_channels, out_channels, kernel_size=1, stride=stride, bias=False,
                                   norm=_norm(norm, out_channels)) if in_channels != out_channels else None)
        s1, s3 = (stride, 1) if stride_in_1x1 else (1, stride)
        self.conv1 = _ConvNorm(in_channels, bottleneck_channels, kernel_size=1, stride=s1, bias=False,
                               norm=_norm(norm, bottleneck_channels))
        self.conv2 = _ConvNorm(bottleneck_channels, bottleneck_channels, kernel_size=3, stride=s3, padding=1,
                               bias=False, norm=_norm(norm, bottleneck_channels))
        self.conv3 = _ConvNorm(bottleneck_channels, out_channels, kernel_size=1, bias=False,
                               norm=_norm(norm, out_channels))

    def forward(self, x):
        out = F.relu_(self.conv1(x))
        out = F.relu_(self.conv2(out))
        out = self.conv3(out)
        out = out + (self.shortcut(x) if self.shortcut is not None else x)
        return F.relu_(out)


class ResNet(nn.Module):
    """Stem + res2..res5; forward returns {name: feature} for ``out_features``.  ``freeze_at`` = 1
    freezes the stem (k = 2 .. 5 would also freeze res2 .. res(k)), as detectron2's freeze()."""

    def __init__(self, stem, stages, out_features=None, freeze_at=0):
        super().__init__()
        self.stem = stem
        self.stage_names = []
        for i, blocks in enumerate(stages):
            name = f"res{i + 2}"
            self.add_module(name, nn.Sequential(*blocks))
            self.stage_names.append(name)
        self.out_features = list(out_features or self.stage_names[-1:])
        self._out_feature_channels = {f"res{i + 2}": s[-1].out_channels for i, s in enumerate(stages)}
        self._out_feature_strides = {f"res{i + 2}": 4 * 2 ** i for i in range(len(stages))}
        self.freeze(freeze_at)

    def freeze(self, freeze_at=0):
        if freeze_at >= 1:
            for p in self.stem.parameters():
                p.requires_grad_(False)
        for idx, name in enumerate(self.stage_names, start=2):
            if freeze_at >= idx:
                for p in getattr(self, name).parameters():
                    p.requires_grad_(False)
        return self

    def forward(self, x):
        outputs = {}
        x = self.stem(x)
        for name in self.stage_names:
            x = getattr(self, name)(x)
            if name in self.out_features:
                outputs[name] = x
        return outputs

    @staticmethod
    def make_default_stages(depth=50, stride_in_1x1=False, norm="BN", in_channels=64, out_channels=256):
        blocks_per = {50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}[depth]
        stages = []
        for i, n in enumerate(blocks_per):
            stride = 1 if i == 0 else 2
            blocks = []
            for b in range(n):
                blocks.append(BottleneckBlock(in_channels, out_channels, bottleneck_channels=out_channels // 4,
                                              stride=stride if b == 0 else 1, norm=norm,
                                              stride_in_1x1=stride_in_1x1))
                in_channels = out_channels
            stages.append(blocks)
            out_channels *= 2
        return stages
