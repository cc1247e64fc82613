"""vCLR DINO on the MI355X MSDeformAttn kernels (reference
projects/vCLR_deformable_mask/modeling/__init__.py): the deformable transformer, the detector
around it (dino.py: ResNet-50 + ChannelMapper features, contrastive-denoising queries, class /
box / mask heads) and its criterion (dn_criterion.py / two_stage_criterion.py).
``attach_detection_heads`` restates the part of ``DINO.__init__`` (dino.py:185-230) that the
transformer's two-stage selection and box refinement read, for the transformer-only bench.
"""
import copy
import math

import torch.nn as nn

from detrex.layers import MLP

from .consistency import ConsisCriterion
from .criterion import DINOCriterion
from .dino import DINO
from .dino_transformer import DINOTransformer, DINOTransformerDecoder, DINOTransformerEncoder


def attach_detection_heads(transformer: DINOTransformer, num_classes: int = 1, embed_dim: int = 256):
    """Per-layer class / box heads (+1 for the encoder proposals) shared with the decoder, with
    DINO's initialisation: prior-probability class bias, zeroed last box layer (dino.py:185-230)."""
    class_embed = nn.Linear(embed_dim, num_classes)
    bbox_embed = MLP(embed_dim, embed_dim, 4, 3)
    class_embed.bias.data.fill_(-math.log((1 - 0.01) / 0.01))
    nn.init.constant_(bbox_embed.layers[-1].weight.data, 0)
    nn.init.constant_(bbox_embed.layers[-1].bias.data, 0)
    n = transformer.decoder.num_layers + 1
    transformer.decoder.class_embed = nn.ModuleList(copy.deepcopy(class_embed) for _ in range(n))
    transformer.decoder.bbox_embed = nn.ModuleList(copy.deepcopy(bbox_embed) for _ in range(n))
    return transformer


__all__ = ["DINOTransformerEncoder", "DINOTransformerDecoder", "DINOTransformer", "attach_detection_heads", "DINO",
           "DINOCriterion", "ConsisCriterion"]
