"""Shared definition of the training-step fixtures (TEST INFRASTRUCTURE).

The benchmarked path (bench.py: CMNeXt in training mode, TRAIN_TYPE Adapter, MMST loss of
train_mm.py:133-148) with its random draws switched off, so that the reference (CPU fp32,
oracle/gen_golden.py) and the product (GPU, bf16 autocast, fused stages, graph replay,
tests/test_gpu_train_parity.py) compute the same function:

  * apply_mask skipped: only the SwinTransformer object is put in eval mode
    (swin.py:1433-1434 tests ``self.training``); every submodule stays in training mode;
  * DropPath p = 0 (drop_path_rate linspace(0, 0.3), swin.py:1252-1255);
  * the Adapters' hard-coded F.dropout(p=0.1, training=self.training) (swin.py:496) off by
    putting the Adapter modules in eval mode;
  * the heads' Dropout2d(0.1) (segformer.py:36) at p = 0.
BatchNorm keeps its training-mode batch statistics (heads' linear_fuse, DAttn fuse_q).
"""
import zlib

import numpy as np
import torch.nn as nn

from fill import seeded

TRAIN_FIXTURES = {
    # tag: (backbone, n_cls, B, H, W, fill seed, input seed)
    "c2_swinb_512": ("SwinTransformer-B", 40, 2, 512, 512, 41, 200),      # C2 geometry (NYU, 512²)
    "c1_swinb_480x640": ("SwinTransformer-B", 40, 2, 480, 640, 43, 210),  # C1 geometry (nyu_rgbd.yaml:19,46)
    "c4_swinl_480x640": ("SwinTransformer-L", 9, 2, 480, 640, 47, 220),   # C4 geometry (MFNet RGB-T, Swin-L)
}
FULL_GRAD_KEYS = ("decode_head.linear_pred.weight", "decode_head.linear_pred.bias",
                  "decode_head_rgb.linear_pred.weight", "decode_head_dte.linear_pred.bias",
                  "backbone.stages.0.blocks.0.MLP_RGB_Adapter.D_fc1.weight",
                  "backbone.stages.0.blocks.1.MLP_DTE_Adapter.D_fc2.weight",
                  "backbone.stages.3.blocks.1.MLP_RGB_Adapter.D_fc2.bias",
                  "backbone.MPGBlocks.0.U_fc1.weight", "backbone.MPGBlocks.2.tfts_gamma_dte",
                  "backbone.DeformMPGBlocks.0.D_fc1.weight", "backbone.DeformMPGBlocks.0.U_fc1.bias",
                  "backbone.DeformMPGBlocks.1.deform_atten.rpe_table",
                  "backbone.DeformMPGBlocks.3.deform_atten.conv_offset_x.0.weight",
                  "backbone.extra_patch_embed.projection.weight")
N_PROJ = 2  # seeded N(0,1) projections per gradient tensor: |<g - g', r>| ~ ||g - g'||


def adapter_trainable(name):
    # optimizers.py:10-20 (TRAIN_TYPE: Adapter)
    return ("Adapter" in name) or ("extra_patch_embed" in name) or ("head" in name) or ("MPG" in name)


def proj_seed(name, j):
    return (zlib.crc32(name.encode()) + 7919 * (j + 1)) & 0x7FFFFFFF


def projection(name, g64, j):
    return float((g64 * seeded(g64.shape, proj_seed(name, j), dtype=np.float64)).sum())


def train_inputs(B, H, W, n_cls, seed):
    """RGB N(0,1) (post-Normalize), depth U[0,1) (/255 only), labels U{0..n_cls-1} with ~10 %
    ignore = 255 (SURVEY §8(d) synthetic inputs)."""
    rgb = seeded((B, 3, H, W), seed)
    dep = seeded((B, 3, H, W), seed + 1, "uniform")
    lbl = (seeded((B, H, W), seed + 2, "uniform") * n_cls).astype(np.int64).clip(0, n_cls - 1)
    lbl[seeded((B, H, W), seed + 3, "uniform") < 0.1] = 255
    return rgb, dep, lbl


def deterministic_train_mode(model):
    model.train()
    model.backbone.training = False  # skip apply_mask only
    for m in model.modules():
        if type(m).__name__ in ("DropPath", "_DropPath"):
            for attr in ("drop_prob", "p"):
                if hasattr(m, attr):
                    setattr(m, attr, 0.0)
        if type(m).__name__ == "Adapter":
            m.training = False
        if isinstance(m, nn.Dropout2d):
            m.p = 0.0
    return model
