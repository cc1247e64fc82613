"""Multi-head self attention with identity and position embeddings
(reference detrex/layers/attention.py:32-140).

A thin wrapper of ``torch.nn.MultiheadAttention`` exactly as the reference has it: the query
(and key) get their position embeddings added, the value does not, and the output is
``identity + proj_drop(attn(...))``.  On ROCm the fused path of ``nn.MultiheadAttention``
dispatches to PyTorch's own flash / memory-efficient kernels; the DINO decoder self-attention
(≈2 200 queries, 8 heads of 32) is a small share of the decoder next to MSDA.
"""
import warnings
from typing import Optional

import torch
import torch.nn as nn


class MultiheadAttention(nn.Module):
    def __init__(self, embed_dim: int, num_heads: int, attn_drop: float = 0.0, proj_drop: float = 0.0,
                 batch_first: bool = False, **kwargs):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.batch_first = batch_first
        self.attn = nn.MultiheadAttention(embed_dim=embed_dim, num_heads=num_heads, dropout=attn_drop,
                                          batch_first=batch_first, **kwargs)
        self.proj_drop = nn.Dropout(proj_drop)

    def forward(self, query: torch.Tensor, key: Optional[torch.Tensor] = None, value: Optional[torch.Tensor] = None,
                identity: Optional[torch.Tensor] = None, query_pos: Optional[torch.Tensor] = None,
                key_pos: Optional[torch.Tensor] = None, attn_mask: Optional[torch.Tensor] = None,
                key_padding_mask: Optional[torch.Tensor] = None, **kwargs) -> torch.Tensor:
        key = query if key is None else key
        value = key if value is None else value
        identity = query if identity is None else identity
        if key_pos is None and query_pos is not None:
            if query_pos.shape == key.shape:
                key_pos = query_pos
            else:
                warnings.warn(f"position encoding of key is missing in {self.__class__.__name__}.")
        if query_pos is not None:
            query = query + query_pos
        if key_pos is not None:
            key = key + key_pos
        out = self.attn(query=query, key=key, value=value, attn_mask=attn_mask,
                        key_padding_mask=key_padding_mask)[0]
        return identity + self.proj_drop(out)
