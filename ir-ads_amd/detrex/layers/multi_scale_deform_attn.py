"""Multi-scale deformable attention (reference detrex/layers/multi_scale_deform_attn.py).

``MultiScaleDeformableAttnFunction`` keeps the reference's autograd signature
(apply(value, spatial_shapes, level_start_index, sampling_locations, attention_weights,
im2col_step) -> grads (grad_value, None, None, grad_loc, grad_aw, None)) on top of the
gfx950 kernels of libirads.so instead of detrex._C.  The module's projections stay on
hipBLASLt.  GPU tensors only: the reference's CPU branch (:341-353) is the oracle's job
(oracle/irads_ref.py), so CPU inputs raise here instead of silently falling back.
"""
import math
import warnings
from typing import Optional

import torch
import torch.nn as nn
from torch.nn.init import constant_, xavier_uniform_

from irads import ops


def _is_power_of_2(n):
    if (not isinstance(n, int)) or (n < 0):
        raise ValueError("invalid input for _is_power_of_2: {} (type: {})".format(n, type(n)))
    return (n & (n - 1) == 0) and n != 0


MultiScaleDeformableAttnFunction = ops.MSDAFn


def multi_scale_deformable_attn_pytorch(value, value_spatial_shapes, sampling_locations, attention_weights):
    """Same contract as the reference helper; runs the HIP kernel (GPU tensors)."""
    lsi = torch.cat([value_spatial_shapes.new_zeros(1), value_spatial_shapes.prod(1).cumsum(0)[:-1]])
    return ops.MSDAFn.apply(value.contiguous(), value_spatial_shapes.contiguous(), lsi.contiguous(),
                            sampling_locations.contiguous(), attention_weights.contiguous(), 64)


class MultiScaleDeformableAttention(nn.Module):
    """Deformable-DETR MSDA module (reference :139-363), same arguments and keys."""

    def __init__(self, embed_dim: int = 256, num_heads: int = 8, num_levels: int = 4, num_points: int = 4,
                 img2col_step: int = 64, dropout: float = 0.1, batch_first: bool = False):
        super().__init__()
        if embed_dim % num_heads != 0:
            raise ValueError("embed_dim must be divisible by num_heads, but got {} and {}".format(embed_dim, num_heads))
        head_dim = embed_dim // num_heads
        self.dropout = nn.Dropout(dropout)
        self.batch_first = batch_first
        if not _is_power_of_2(head_dim):
            warnings.warn("You'd better set d_model in MSDeformAttn to make sure that each dim of the attention "
                          "head a power of 2, which is more efficient.")
        self.im2col_step = img2col_step
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.num_levels = num_levels
        self.num_points = num_points
        self.sampling_offsets = nn.Linear(embed_dim, num_heads * num_levels * num_points * 2)
        self.attention_weights = nn.Linear(embed_dim, num_heads * num_levels * num_points)
        self.value_proj = nn.Linear(embed_dim, embed_dim)
        self.output_proj = nn.Linear(embed_dim, embed_dim)
        self.init_weights()

    def init_weights(self):
        constant_(self.sampling_offsets.weight.data, 0.0)
        thetas = torch.arange(self.num_heads, dtype=torch.float32) * (2.0 * math.pi / self.num_heads)
        grid = torch.stack([thetas.cos(), thetas.sin()], -1)
        grid = (grid / grid.abs().max(-1, keepdim=True)[0]).view(self.num_heads, 1, 1, 2)
        grid = grid.repeat(1, self.num_levels, self.num_points, 1)
        for i in range(self.num_points):
            grid[:, :, i, :] *= i + 1
        with torch.no_grad():
            self.sampling_offsets.bias = nn.Parameter(grid.view(-1))
        constant_(self.attention_weights.weight.data, 0.0)
        constant_(self.attention_weights.bias.data, 0.0)
        xavier_uniform_(self.value_proj.weight.data)
        constant_(self.value_proj.bias.data, 0.0)
        xavier_uniform_(self.output_proj.weight.data)
        constant_(self.output_proj.bias.data, 0.0)

    def forward(self, query: torch.Tensor, key: Optional[torch.Tensor] = None, value: Optional[torch.Tensor] = None,
                identity: Optional[torch.Tensor] = None, query_pos: Optional[torch.Tensor] = None,
                key_padding_mask: Optional[torch.Tensor] = None, reference_points: Optional[torch.Tensor] = None,
                spatial_shapes: Optional[torch.Tensor] = None, level_start_index: Optional[torch.Tensor] = None,
                **kwargs) -> torch.Tensor:
        if value is None:
            value = query
        if identity is None:
            identity = query
        if query_pos is not None:
            query = query + query_pos
        if not self.batch_first:
            query = query.permute(1, 0, 2)
            value = value.permute(1, 0, 2)
        bs, num_query, _ = query.shape
        _, num_value, _ = value.shape
        assert (spatial_shapes[:, 0] * spatial_shapes[:, 1]).sum() == num_value
        M, L, P = self.num_heads, self.num_levels, self.num_points
        value = self.value_proj(value)
        if key_padding_mask is not None:
            value = value.masked_fill(key_padding_mask[..., None], float(0))
        value = value.view(bs, num_value, M, -1)
        offsets = self.sampling_offsets(query).view(bs, num_query, M, L, P, 2)
        weights = self.attention_weights(query).view(bs, num_query, M, L * P).softmax(-1)
        weights = weights.view(bs, num_query, M, L, P)
        if reference_points.shape[-1] == 2:
            normalizer = torch.stack([spatial_shapes[..., 1], spatial_shapes[..., 0]], -1)
            loc = reference_points[:, :, None, :, None, :] + offsets / normalizer[None, None, None, :, None, :]
        elif reference_points.shape[-1] == 4:
            loc = (reference_points[:, :, None, :, None, :2]
                   + offsets / P * reference_points[:, :, None, :, None, 2:] * 0.5)
        else:
            raise ValueError("Last dim of reference_points must be 2 or 4, but get {} instead.".format(
                reference_points.shape[-1]))
        in_dtype = value.dtype
        # the kernel computes in fp32 (fp16/bf16 are upcast, as the reference does for fp16, :343)
        kdt = torch.float64 if in_dtype == torch.float64 else torch.float32
        if not value.is_cuda:
            raise RuntimeError("MultiScaleDeformableAttention: the MI355X path runs on GPU tensors only")
        output = ops.MSDAFn.apply(value.to(kdt).contiguous(), spatial_shapes.contiguous(),
                                  level_start_index.contiguous(), loc.to(kdt).contiguous(),
                                  weights.to(kdt).contiguous(), self.im2col_step)
        if in_dtype == torch.float16:
            output = output.to(torch.float16)
        output = self.output_proj(output)
        if not self.batch_first:
            output = output.permute(1, 0, 2)
        return self.dropout(output) + identity
