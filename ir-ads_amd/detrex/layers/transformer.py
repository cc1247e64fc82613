"""Transformer layer containers (reference detrex/layers/transformer.py:33-228).

``BaseTransformerLayer`` runs an ``operation_order`` over attention / norm / FFN modules
with the reference's identity bookkeeping: after every attention the running ``identity``
becomes that attention's output, and in pre-norm mode (order starting with ``"norm"``) the
identity is handed to the attention / FFN explicitly.  ``TransformerLayerSequence`` deep-copies
one layer ``num_layers`` times.  Keys match the reference (``attentions.*``, ``ffns.*``,
``norms.*``, ``layers.*``), so reference state dicts load unchanged.
"""
import copy
import warnings
from typing import List

import torch
import torch.nn as nn


class BaseTransformerLayer(nn.Module):
    """Reference transformer.py:33-173 (same arguments, same attribute names)."""

    def __init__(self, attn, ffn: nn.Module, norm: nn.Module, operation_order: tuple = None):
        super().__init__()
        assert set(operation_order).issubset({"self_attn", "norm", "cross_attn", "ffn"})
        num_attn = sum(op in ("self_attn", "cross_attn") for op in operation_order)
        if isinstance(attn, nn.Module):
            attn = [copy.deepcopy(attn) for _ in range(num_attn)]
        elif len(attn) != num_attn:
            raise AssertionError(f"The length of attn (nn.Module or List[nn.Module]) {num_attn}"
                                 f"is not consistent with the number of attention in "
                                 f"operation_order {operation_order}")
        self.num_attn = num_attn
        self.operation_order = operation_order
        self.pre_norm = operation_order[0] == "norm"
        self.attentions = nn.ModuleList(attn)
        self.embed_dim = self.attentions[0].embed_dim
        self.ffns = nn.ModuleList(copy.deepcopy(ffn) for _ in range(operation_order.count("ffn")))
        self.norms = nn.ModuleList(copy.deepcopy(norm) for _ in range(operation_order.count("norm")))

    def forward(self, query: torch.Tensor, key: torch.Tensor = None, value: torch.Tensor = None,
                query_pos: torch.Tensor = None, key_pos: torch.Tensor = None,
                attn_masks: List[torch.Tensor] = None, query_key_padding_mask: torch.Tensor = None,
                key_padding_mask: torch.Tensor = None, **kwargs):
        if attn_masks is None:
            attn_masks = [None] * self.num_attn
        elif isinstance(attn_masks, torch.Tensor):
            warnings.warn(f"Use same attn_mask in all attentions in {self.__class__.__name__} ")
            attn_masks = [attn_masks] * self.num_attn
        elif len(attn_masks) != self.num_attn:
            raise AssertionError(f"The length of attn_masks {len(attn_masks)} must be equal to the number of "
                                 f"attention in operation_order {self.num_attn}")
        identity = query
        ai = ni = fi = 0
        for op in self.operation_order:
            if op == "norm":
                query = self.norms[ni](query)
                ni += 1
            elif op == "ffn":
                query = self.ffns[fi](query, identity if self.pre_norm else None)
                fi += 1
            else:
                self_attn = op == "self_attn"
                query = self.attentions[ai](
                    query, query if self_attn else key, query if self_attn else value,
                    identity if self.pre_norm else None,
                    query_pos=query_pos, key_pos=query_pos if self_attn else key_pos,
                    attn_mask=attn_masks[ai],
                    key_padding_mask=query_key_padding_mask if self_attn else key_padding_mask,
                    **kwargs)
                ai += 1
                identity = query
        return query


class TransformerLayerSequence(nn.Module):
    """Reference transformer.py:176-228: ``num_layers`` deep copies of one layer."""

    def __init__(self, transformer_layers=None, num_layers=None):
        super().__init__()
        self.num_layers = num_layers
        self.layers = nn.ModuleList()
        if isinstance(transformer_layers, nn.Module):
            for _ in range(num_layers):
                self.layers.append(copy.deepcopy(transformer_layers))
        else:
            assert isinstance(transformer_layers, list) and len(transformer_layers) == num_layers

    def forward(self):
        raise NotImplementedError()
