"""SegFormer decode head (reference semseg/models/heads/segformer.py:7-48)."""
from typing import Tuple

import torch
from torch import nn, Tensor
from torch.nn import functional as F

from irads import ops
from semseg.models.layers.common import TrainLinear


class MLP(nn.Module):
    def __init__(self, dim, embed_dim):
        super().__init__()
        self.proj = TrainLinear(dim, embed_dim)

    def forward(self, x: Tensor) -> Tensor:
        return self.proj(x.flatten(2).transpose(1, 2))


class ConvModule(nn.Module):
    def __init__(self, c1, c2):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, 1, bias=False)
        self.bn = nn.BatchNorm2d(c2)  # per-GPU BN, as the reference (no SyncBN)
        self.activate = nn.ReLU(True)

    def forward(self, x: Tensor) -> Tensor:
        return self.activate(self.bn(self.conv(x)))


class SegFormerHead(nn.Module):
    def __init__(self, dims: list, embed_dim: int = 256, num_classes: int = 19):
        super().__init__()
        for i, dim in enumerate(dims):
            self.add_module(f"linear_c{i + 1}", MLP(dim, embed_dim))
        self.linear_fuse = ConvModule(embed_dim * 4, embed_dim)
        self.linear_pred = nn.Conv2d(embed_dim, num_classes, 1)
        self.dropout = nn.Dropout2d(0.1)

    def forward(self, features: Tuple[Tensor, Tensor, Tensor, Tensor]) -> Tensor:
        B, _, H, W = features[0].shape
        outs = [self.linear_c1(features[0]).permute(0, 2, 1).reshape(B, -1, H, W)]
        for i, f in enumerate(features[1:]):
            cf = getattr(self, f"linear_c{i + 2}")(f).permute(0, 2, 1).reshape(B, -1, *f.shape[-2:])
            outs.append(ops.resize(cf, (H, W)))  # F.interpolate(bilinear, align_corners=False)
        seg = self.linear_fuse(torch.cat(outs[::-1], dim=1))
        return self.linear_pred(self.dropout(seg))
