"""Seeded inputs of the reduced vCLR DINO transformer case (TEST INFRASTRUCTURE).

Shared by the fixture generator (oracle/gen_golden.py, reference side) and the GPU parity test
(tests/test_gpu_dino.py, product side) so both build bit-identical inputs from the seeds.
"""
import numpy as np
import torch

from fill import seeded


def t(a, dtype=None):
    x = torch.from_numpy(np.ascontiguousarray(a))
    return x.to(dtype) if dtype is not None else x


DINO_LEVELS = [(10, 14), (5, 7), (3, 4), (2, 2)]
DINO_BS, DINO_DN, DINO_PROPOSALS, DINO_LAYERS = 2, 10, 30, 6


def dino_inputs(dtype=torch.float64):
    """Seeded C5-shaped (reduced) inputs: 4 levels, image 1 padded to ~70 % x 80 % of each level,
    10 denoising queries in 2 groups plus 30 two-stage proposals (dn_components.py layout)."""
    feats, masks = [], []
    for lvl, (H, W) in enumerate(DINO_LEVELS):
        feats.append(t(seeded((DINO_BS, 256, H, W), 41 + lvl), dtype))
        m = torch.zeros(DINO_BS, H, W, dtype=torch.bool)
        m[1, -(-7 * H // 10):, :] = True  # valid rows ceil(0.7 H), columns ceil(0.8 W)
        m[1, :, -(-8 * W // 10):] = True
        masks.append(m)
    dn_label = t(seeded((DINO_BS, DINO_DN, 256), 51), dtype)
    dn_box = t(seeded((DINO_BS, DINO_DN, 4), 52), dtype)
    n = DINO_DN + DINO_PROPOSALS
    attn = torch.zeros(n, n, dtype=torch.bool)
    attn[DINO_DN:, :DINO_DN] = True
    half = DINO_DN // 2
    attn[:half, half:DINO_DN] = True
    attn[half:DINO_DN, :half] = True
    return feats, masks, dn_label, dn_box, attn
