from .multi_scale_deform_attn import (MultiScaleDeformableAttention, MultiScaleDeformableAttnFunction,
                                      multi_scale_deformable_attn_pytorch)

__all__ = ['MultiScaleDeformableAttention', 'MultiScaleDeformableAttnFunction', 'multi_scale_deformable_attn_pytorch']
