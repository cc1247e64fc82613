"""Small building blocks (reference semseg/models/layers/common.py)."""
import torch
from torch import nn, Tensor


class ConvModule(nn.Sequential):
    def __init__(self, c1, c2, k, s=1, p=0, d=1, g=1):
        super().__init__(nn.Conv2d(c1, c2, k, s, p, d, g, bias=False), nn.BatchNorm2d(c2), nn.ReLU(True))


class DropPath(nn.Module):
    """Stochastic depth per sample: x / keep * floor(keep + U[0, 1))."""

    def __init__(self, p: float = None):
        super().__init__()
        self.p = p

    def forward(self, x: Tensor) -> Tensor:
        if not self.p or not self.training:
            return x
        keep = 1 - self.p
        mask = (keep + torch.rand((x.shape[0],) + (1,) * (x.ndim - 1), dtype=x.dtype, device=x.device)).floor_()
        return x.div(keep) * mask
