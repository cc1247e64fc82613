"""DINO deformable transformer of the vCLR detector
(reference projects/vCLR_deformable_mask/modeling/dino_transformer.py:32-475).

This is the caller side of MSDeformAttn at configuration C5: a 6-layer encoder whose
self-attention is ``MultiScaleDeformableAttention`` over all 4 levels (Q = S ≈ 22 k tokens per
image at 800×1333) and a 6-layer decoder with query self-attention followed by MSDA
cross-attention of ≈2 200 queries into the encoder memory (4-d reference boxes).  Both MSDA
call sites run the gfx950 kernels of ``libirads.so`` (``irads_msda_fwd`` and the atomic-free
``irads_msda_bwd_gather``); projections and norms stay on hipBLASLt / PyTorch.

Same constructor arguments, forward contract and state-dict keys as the reference.
``use_checkpoint`` is accepted and, as in the reference (:74-77, :160-163, where
``checkpoint_wrapper`` only rebinds the loop variable), changes nothing.
"""
import torch
import torch.nn as nn

from detrex.layers import (FFN, MLP, BaseTransformerLayer, MultiheadAttention, MultiScaleDeformableAttention,
                           TransformerLayerSequence, get_sine_pos_embed)
from detrex.utils import inverse_sigmoid


class DINOTransformerEncoder(TransformerLayerSequence):
    """Reference dino_transformer.py:32-104: post-norm (attn, norm, ffn, norm) x num_layers."""

    def __init__(self, embed_dim: int = 256, num_heads: int = 8, feedforward_dim: int = 1024,
                 attn_dropout: float = 0.1, ffn_dropout: float = 0.1, num_layers: int = 6,
                 post_norm: bool = False, num_feature_levels: int = 4, use_checkpoint: bool = False):
        layer = BaseTransformerLayer(
            attn=MultiScaleDeformableAttention(embed_dim=embed_dim, num_heads=num_heads, dropout=attn_dropout,
                                               batch_first=True, num_levels=num_feature_levels),
            ffn=FFN(embed_dim=embed_dim, feedforward_dim=feedforward_dim, output_dim=embed_dim, num_fcs=2,
                    ffn_drop=ffn_dropout),
            norm=nn.LayerNorm(embed_dim),
            operation_order=("self_attn", "norm", "ffn", "norm"))
        super().__init__(transformer_layers=layer, num_layers=num_layers)
        self.embed_dim = self.layers[0].embed_dim
        self.pre_norm = self.layers[0].pre_norm
        self.post_norm_layer = nn.LayerNorm(self.embed_dim) if post_norm else None

    def forward(self, query, key, value, query_pos=None, key_pos=None, attn_masks=None,
                query_key_padding_mask=None, key_padding_mask=None, **kwargs):
        for layer in self.layers:
            query = layer(query, key, value, query_pos=query_pos, attn_masks=attn_masks,
                          query_key_padding_mask=query_key_padding_mask, key_padding_mask=key_padding_mask,
                          **kwargs)
        return query if self.post_norm_layer is None else self.post_norm_layer(query)


class DINOTransformerDecoder(TransformerLayerSequence):
    """Reference dino_transformer.py:107-240: (self_attn, norm, cross_attn, norm, ffn, norm) x
    num_layers with iterative box refinement; ``class_embed`` / ``bbox_embed`` are attached by
    the detector (reference dino.py:225-226)."""

    def __init__(self, embed_dim: int = 256, num_heads: int = 8, feedforward_dim: int = 1024,
                 attn_dropout: float = 0.1, ffn_dropout: float = 0.1, num_layers: int = 6,
                 return_intermediate: bool = True, num_feature_levels: int = 4, look_forward_twice: bool = True,
                 use_checkpoint: bool = True):
        layer = BaseTransformerLayer(
            attn=[MultiheadAttention(embed_dim=embed_dim, num_heads=num_heads, attn_drop=attn_dropout,
                                     batch_first=True),
                  MultiScaleDeformableAttention(embed_dim=embed_dim, num_heads=num_heads, dropout=attn_dropout,
                                                batch_first=True, num_levels=num_feature_levels)],
            ffn=FFN(embed_dim=embed_dim, feedforward_dim=feedforward_dim, output_dim=embed_dim,
                    ffn_drop=ffn_dropout),
            norm=nn.LayerNorm(embed_dim),
            operation_order=("self_attn", "norm", "cross_attn", "norm", "ffn", "norm"))
        super().__init__(transformer_layers=layer, num_layers=num_layers)
        self.return_intermediate = return_intermediate
        self.ref_point_head = MLP(2 * embed_dim, embed_dim, embed_dim, 2)
        self.bbox_embed = None
        self.class_embed = None
        self.look_forward_twice = look_forward_twice
        self.norm = nn.LayerNorm(embed_dim)

    def forward(self, query, key, value, query_pos=None, key_pos=None, attn_masks=None,
                query_key_padding_mask=None, key_padding_mask=None, reference_points=None, valid_ratios=None,
                **kwargs):
        output = query
        bs = output.shape[0]
        if reference_points.dim() == 2:
            reference_points = reference_points.unsqueeze(0).repeat(bs, 1, 1)
        boxes = reference_points.shape[-1] == 4
        assert boxes or reference_points.shape[-1] == 2
        # per-level scaling of the normalised references by the valid-area ratios
        ratio = torch.cat([valid_ratios, valid_ratios], -1) if boxes else valid_ratios
        states, refs = [], []
        new_reference_points = reference_points
        for idx, layer in enumerate(self.layers):
            ref_input = reference_points[:, :, None] * ratio[:, None]
            query_sine_embed = get_sine_pos_embed(ref_input[:, :, 0, :])
            query_pos = self.ref_point_head(query_sine_embed)
            output = layer(output, key, value, query_pos=query_pos, key_pos=key_pos,
                           query_sine_embed=query_sine_embed, attn_masks=attn_masks,
                           query_key_padding_mask=query_key_padding_mask, key_padding_mask=key_padding_mask,
                           reference_points=ref_input, **kwargs)
            if self.bbox_embed is not None:
                delta = self.bbox_embed[idx](output)
                if boxes:
                    new_reference_points = (delta + inverse_sigmoid(reference_points)).sigmoid()
                else:
                    new_reference_points = delta
                    new_reference_points[..., :2] = delta[..., :2] + inverse_sigmoid(reference_points)
                    new_reference_points = new_reference_points.sigmoid()
                reference_points = new_reference_points.detach()
            if self.return_intermediate:
                states.append(self.norm(output))
                refs.append(new_reference_points if self.look_forward_twice else reference_points)
        if self.return_intermediate:
            return torch.stack(states), torch.stack(refs)
        return output, reference_points


class DINOTransformer(nn.Module):
    """Reference dino_transformer.py:243-475: level embeddings, encoder, two-stage proposal
    selection (top-k of the encoder class scores), decoder."""

    def __init__(self, encoder=None, decoder=None, num_feature_levels=4, two_stage_num_proposals=900,
                 learnt_init_query=True):
        super().__init__()
        self.encoder = encoder
        self.decoder = decoder
        self.num_feature_levels = num_feature_levels
        self.two_stage_num_proposals = two_stage_num_proposals
        self.embed_dim = self.encoder.embed_dim
        self.level_embeds = nn.Parameter(torch.Tensor(self.num_feature_levels, self.embed_dim))
        self.learnt_init_query = learnt_init_query
        if self.learnt_init_query:
            self.tgt_embed = nn.Embedding(self.two_stage_num_proposals, self.embed_dim)
        self.enc_output = nn.Linear(self.embed_dim, self.embed_dim)
        self.enc_output_norm = nn.LayerNorm(self.embed_dim)
        self.init_weights()

    def init_weights(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)
        for m in self.modules():
            if isinstance(m, MultiScaleDeformableAttention):
                m.init_weights()
        nn.init.normal_(self.level_embeds)

    def gen_encoder_output_proposals(self, memory, memory_padding_mask, spatial_shapes):
        """Reference :281-317: one (cx, cy, w, h) anchor per memory token, in logit space;
        padded or near-border tokens get +inf and a zeroed memory row."""
        N = memory.shape[0]
        proposals, start = [], 0
        for lvl, (H, W) in enumerate(spatial_shapes.tolist()):
            pad = memory_padding_mask[:, start:start + H * W].view(N, H, W)
            valid_h = (~pad[:, :, 0]).sum(1)
            valid_w = (~pad[:, 0, :]).sum(1)
            gy, gx = torch.meshgrid(torch.linspace(0, H - 1, H, dtype=torch.float32, device=memory.device),
                                    torch.linspace(0, W - 1, W, dtype=torch.float32, device=memory.device),
                                    indexing="ij")
            grid = torch.stack([gx, gy], -1)
            scale = torch.stack([valid_w, valid_h], 1).view(N, 1, 1, 2)
            grid = (grid.unsqueeze(0).expand(N, -1, -1, -1) + 0.5) / scale
            wh = torch.ones_like(grid) * 0.05 * (2.0 ** lvl)
            proposals.append(torch.cat((grid, wh), -1).view(N, -1, 4))
            start += H * W
        props = torch.cat(proposals, 1)
        valid = ((props > 0.01) & (props < 0.99)).all(-1, keepdim=True)
        props = torch.log(props / (1 - props))
        props = props.masked_fill(memory_padding_mask.unsqueeze(-1), float("inf"))
        props = props.masked_fill(~valid, float("inf"))
        out = memory.masked_fill(memory_padding_mask.unsqueeze(-1), 0.0).masked_fill(~valid, 0.0)
        return self.enc_output_norm(self.enc_output(out)), props

    @staticmethod
    def get_reference_points(spatial_shapes, valid_ratios, device):
        """Reference :319-352: pixel-centre references of every level, scaled by the valid ratios."""
        refs = []
        for lvl, (H, W) in enumerate(spatial_shapes.tolist()):
            ry, rx = torch.meshgrid(torch.linspace(0.5, H - 0.5, H, dtype=torch.float32, device=device),
                                    torch.linspace(0.5, W - 0.5, W, dtype=torch.float32, device=device),
                                    indexing="ij")
            ry = ry.reshape(-1)[None] / (valid_ratios[:, None, lvl, 1] * H)
            rx = rx.reshape(-1)[None] / (valid_ratios[:, None, lvl, 0] * W)
            refs.append(torch.stack((rx, ry), -1))
        return torch.cat(refs, 1)[:, :, None] * valid_ratios[:, None]

    def get_valid_ratio(self, mask):
        _, H, W = mask.shape
        vh = (~mask[:, :, 0]).sum(1).float() / H
        vw = (~mask[:, 0, :]).sum(1).float() / W
        return torch.stack([vw, vh], -1)

    def forward(self, multi_level_feats, multi_level_masks, multi_level_pos_embeds, query_embed, attn_masks,
                **kwargs):
        feats, masks, pos, shapes = [], [], [], []
        for lvl, (feat, mask, pe) in enumerate(zip(multi_level_feats, multi_level_masks, multi_level_pos_embeds)):
            shapes.append(tuple(feat.shape[2:]))
            feats.append(feat.flatten(2).transpose(1, 2))
            masks.append(mask.flatten(1))
            pos.append(pe.flatten(2).transpose(1, 2) + self.level_embeds[lvl].view(1, 1, -1))
        feat_flatten = torch.cat(feats, 1)
        mask_flatten = torch.cat(masks, 1)
        lvl_pos_embed_flatten = torch.cat(pos, 1)
        spatial_shapes = torch.as_tensor(shapes, dtype=torch.long, device=feat_flatten.device)
        level_start_index = torch.cat((spatial_shapes.new_zeros((1,)), spatial_shapes.prod(1).cumsum(0)[:-1]))
        valid_ratios = torch.stack([self.get_valid_ratio(m) for m in multi_level_masks], 1)
        reference_points = self.get_reference_points(spatial_shapes, valid_ratios, device=feat_flatten.device)

        memory = self.encoder(query=feat_flatten, key=None, value=None, query_pos=lvl_pos_embed_flatten,
                              query_key_padding_mask=mask_flatten, spatial_shapes=spatial_shapes,
                              reference_points=reference_points, level_start_index=level_start_index,
                              valid_ratios=valid_ratios, **kwargs)

        output_memory, output_proposals = self.gen_encoder_output_proposals(memory, mask_flatten, spatial_shapes)
        nl = self.decoder.num_layers
        enc_outputs_class = self.decoder.class_embed[nl](output_memory)
        enc_outputs_coord_unact = self.decoder.bbox_embed[nl](output_memory) + output_proposals
        topk_proposals = torch.topk(enc_outputs_class.max(-1)[0], self.two_stage_num_proposals, dim=1)[1]
        topk_coords_unact = torch.gather(enc_outputs_coord_unact, 1, topk_proposals.unsqueeze(-1).repeat(1, 1, 4))
        reference_points = topk_coords_unact.detach().sigmoid()
        if query_embed[1] is not None:
            reference_points = torch.cat([query_embed[1].sigmoid(), reference_points], 1)
        init_reference_out = reference_points
        target_unact = torch.gather(output_memory, 1,
                                    topk_proposals.unsqueeze(-1).repeat(1, 1, output_memory.shape[-1]))
        bs = feat_flatten.shape[0]
        target = self.tgt_embed.weight[None].repeat(bs, 1, 1) if self.learnt_init_query else target_unact.detach()
        if query_embed[0] is not None:
            target = torch.cat([query_embed[0], target], 1)

        inter_states, inter_references = self.decoder(
            query=target, key=memory, value=memory, query_pos=None, key_padding_mask=mask_flatten,
            reference_points=reference_points, spatial_shapes=spatial_shapes, level_start_index=level_start_index,
            valid_ratios=valid_ratios, attn_masks=attn_masks, **kwargs)
        return (inter_states, init_reference_out, inter_references, target_unact, topk_coords_unact.sigmoid(),
                memory)
