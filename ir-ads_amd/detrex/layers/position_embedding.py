"""Sine position embeddings (reference detrex/layers/position_embedding.py:28-212)."""
import math

import torch
import torch.nn as nn


# The arguments of a fully padded row or column are huge: the normalised cumsum there is
# (0 - 0.5) / (0 + eps) * 2 pi ~ -3e6 (eps = 1e-6), so one ulp of a frequency moves the sine by up to
# 0.2.  The GPU's fp32 pow(T, e) differs from the CPU's (the reference run that made
# tests/golden/dino_detector_step.npz) by an ulp on some frequencies, and its fp32 sin / cos of
# such arguments is not correctly rounded either; the CPU's are (pow exactly, sin / cos within one
# ulp of the fp64 result).  So the frequencies are the fp64 pow rounded to fp32 (bit-identical to
# the CPU's fp32 pow for every T^(2 floor(i/2)/F) used here) and the sines the fp64 sine of the fp32
# argument, rounded (scripts/dino_det_dump.py localised the round-4 DINO detector mismatch here).
def _frequencies(num_pos_feats, temperature, device):
    i = torch.arange(num_pos_feats, dtype=torch.float32, device=device)
    e = 2 * torch.div(i, 2, rounding_mode="floor") / num_pos_feats  # exact in fp32
    return (float(temperature) ** e.double()).float()


def _sin(t):
    return t.double().sin().to(t.dtype) if t.dtype == torch.float32 else t.sin()


def _cos(t):
    return t.double().cos().to(t.dtype) if t.dtype == torch.float32 else t.cos()


class PositionEmbeddingSine(nn.Module):
    """DETR sine embedding of a padding mask (reference position_embedding.py:28-117)."""

    def __init__(self, num_pos_feats: int = 64, temperature: int = 10000, scale: float = 2 * math.pi,
                 eps: float = 1e-6, offset: float = 0.0, normalize: bool = False):
        super().__init__()
        if normalize:
            assert isinstance(scale, (float, int)), ("when normalize is set, scale should be provided and in "
                                                     "float or int type, " f"found {type(scale)}")
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.normalize = normalize
        self.scale = scale
        self.eps = eps
        self.offset = offset

    def forward(self, mask: torch.Tensor, **kwargs) -> torch.Tensor:
        assert mask is not None
        not_mask = ~mask
        y = not_mask.cumsum(1, dtype=torch.float32)
        x = not_mask.cumsum(2, dtype=torch.float32)
        if self.normalize:
            y = (y + self.offset) / (y[:, -1:, :] + self.eps) * self.scale
            x = (x + self.offset) / (x[:, :, -1:] + self.eps) * self.scale
        dim_t = _frequencies(self.num_pos_feats, self.temperature, mask.device)
        px = x[:, :, :, None] / dim_t
        py = y[:, :, :, None] / dim_t
        B, H, W = mask.shape
        px = torch.stack((_sin(px[:, :, :, 0::2]), _cos(px[:, :, :, 1::2])), dim=4).view(B, H, W, -1)
        py = torch.stack((_sin(py[:, :, :, 0::2]), _cos(py[:, :, :, 1::2])), dim=4).view(B, H, W, -1)
        return torch.cat((py, px), dim=3).permute(0, 3, 1, 2)


def get_sine_pos_embed(pos_tensor: torch.Tensor, num_pos_feats: int = 128, temperature: int = 10000,
                       exchange_xy: bool = True) -> torch.Tensor:
    """Sine embedding of each coordinate of ``pos_tensor`` (reference position_embedding.py:178-212).

    Each coordinate c gives ``num_pos_feats`` features: sin of the even and cos of the odd
    frequencies of ``2π·c / T^(2⌊i/2⌋/F)``, interleaved; with ``exchange_xy`` the first two
    coordinates' blocks swap places (``[pos(y), pos(x), ...]``).
    """
    dim_t = _frequencies(num_pos_feats, temperature, pos_tensor.device)
    scale = 2 * math.pi

    def embed(c):
        s = c * scale / dim_t
        return torch.stack((_sin(s[:, :, 0::2]), _cos(s[:, :, 1::2])), dim=3).flatten(2)

    parts = [embed(c) for c in pos_tensor.split([1] * pos_tensor.shape[-1], dim=-1)]
    if exchange_xy:
        parts[0], parts[1] = parts[1], parts[0]
    return torch.cat(parts, dim=2)
