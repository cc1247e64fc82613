"""The vCLR DINO-R50 model as configs/models/dino_r50.py builds it (LazyCall tree restated as one
function): ResNet-50 (FrozenBN, freeze_at 1) -> ChannelMapper (1x1 + GroupNorm(32), 4 outputs)
-> DINOTransformer (6 + 6 layers, d 256, 8 heads, FFN 2048) -> DINO with DINOCriterion (Hungarian
matcher: class 2 / L1 5 / GIoU 2, focal) and the auxiliary / encoder loss weights
(dino_r50.py:138-147).  Layer counts, queries and denoising groups are arguments so tests can
build the reduced case."""
import copy

import torch.nn as nn

from detrex.layers import PositionEmbeddingSine
from detrex.modeling import BasicStem, ChannelMapper, HungarianMatcher, ResNet

from ..modeling.consistency import ConsisCriterion
from ..modeling.criterion import DINOCriterion
from ..modeling.dino import DINO
from ..modeling.dino_transformer import DINOTransformer, DINOTransformerDecoder, DINOTransformerEncoder

BASE_WEIGHTS = {"loss_class": 1, "loss_bbox": 5.0, "loss_giou": 2.0, "loss_class_dn": 0, "loss_bbox_dn": 0.0,
                "loss_giou_dn": 0.0, "loss_mask": 1.0, "loss_dice": 5.0, "loss_mask_dn": 0, "loss_dice_dn": 0}


def weight_dict(dec_layers):
    w = dict(BASE_WEIGHTS)
    w.update({k + "_enc": v for k, v in BASE_WEIGHTS.items()})
    for i in range(dec_layers - 1):
        w.update({k + f"_{i}": v for k, v in BASE_WEIGHTS.items()})
    return w


def build_model(num_classes=80, num_queries=900, enc_layers=6, dec_layers=6, dn_number=100, label_noise_ratio=0.5,
                box_noise_scale=1.0, device="cuda", consistency=True):
    backbone = ResNet(stem=BasicStem(in_channels=3, out_channels=64, norm="FrozenBN"),
                      stages=ResNet.make_default_stages(depth=50, stride_in_1x1=False, norm="FrozenBN"),
                      out_features=["res3", "res4", "res5"], freeze_at=1)
    neck = ChannelMapper(input_shapes={"res3": 512, "res4": 1024, "res5": 2048}, in_features=["res3", "res4", "res5"],
                         out_channels=256, num_outs=4, kernel_size=1,
                         norm_layer=nn.GroupNorm(num_groups=32, num_channels=256))
    transformer = DINOTransformer(
        encoder=DINOTransformerEncoder(embed_dim=256, num_heads=8, feedforward_dim=2048, attn_dropout=0.0,
                                       ffn_dropout=0.0, num_layers=enc_layers, post_norm=False, num_feature_levels=4),
        decoder=DINOTransformerDecoder(embed_dim=256, num_heads=8, feedforward_dim=2048, attn_dropout=0.0,
                                       ffn_dropout=0.0, num_layers=dec_layers, return_intermediate=True,
                                       num_feature_levels=4),
        num_feature_levels=4, two_stage_num_proposals=num_queries)
    matcher = HungarianMatcher(cost_class=2.0, cost_bbox=5.0, cost_giou=2.0, cost_class_type="focal_loss_cost",
                               alpha=0.25, gamma=2.0)
    criterion = DINOCriterion(num_classes=num_classes, matcher=matcher, weight_dict=copy.deepcopy(weight_dict(dec_layers)),
                              loss_class_type="focal_loss", alpha=0.25, gamma=2.0, two_stage_binary_cls=False)
    # the siamese consistency loss with its own matcher (dino_r50.py:110-130); the teacher it compares
    # against is the model's EMA (ema.may_build_model_ema + train_net.run_step's update)
    consis = ConsisCriterion(matcher=HungarianMatcher(cost_class=2.0, cost_bbox=5.0, cost_giou=2.0,
                                                      cost_class_type="focal_loss_cost", alpha=0.25, gamma=2.0),
                             weight_dict=copy.deepcopy(BASE_WEIGHTS)) if consistency else None
    return DINO(backbone=backbone,
                position_embedding=PositionEmbeddingSine(num_pos_feats=128, temperature=10000, normalize=True,
                                                         offset=-0.5),
                neck=neck, transformer=transformer, embed_dim=256, num_classes=num_classes, num_queries=num_queries,
                criterion=criterion, aux_loss=True, dn_number=dn_number, label_noise_ratio=label_noise_ratio,
                box_noise_scale=box_noise_scale, device=device, consistency_criterion=consis)
