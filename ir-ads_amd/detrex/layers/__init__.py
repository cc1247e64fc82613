from .attention import MultiheadAttention
from .box_ops import box_cxcywh_to_xyxy, box_iou, box_xyxy_to_cxcywh, generalized_box_iou
from .mlp import FFN, MLP
from .multi_scale_deform_attn import (MultiScaleDeformableAttention, MultiScaleDeformableAttnFunction,
                                      multi_scale_deformable_attn_pytorch)
from .position_embedding import PositionEmbeddingSine, get_sine_pos_embed
from .transformer import BaseTransformerLayer, TransformerLayerSequence

__all__ = ['MultiScaleDeformableAttention', 'MultiScaleDeformableAttnFunction', 'multi_scale_deformable_attn_pytorch',
           'MultiheadAttention', 'FFN', 'MLP', 'PositionEmbeddingSine', 'get_sine_pos_embed', 'BaseTransformerLayer',
           'TransformerLayerSequence', 'box_cxcywh_to_xyxy', 'box_xyxy_to_cxcywh', 'box_iou', 'generalized_box_iou']
