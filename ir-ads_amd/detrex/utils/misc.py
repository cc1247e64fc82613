"""Box-coordinate helper used by the DINO decoder (reference detrex/utils/misc.py:38-46)."""
import torch


def inverse_sigmoid(x, eps=1e-3):
    """logit(x) with x clamped to [0, 1] and both odds terms floored at ``eps``."""
    x = x.clamp(min=0, max=1)
    return torch.log(x.clamp(min=eps) / (1 - x).clamp(min=eps))
