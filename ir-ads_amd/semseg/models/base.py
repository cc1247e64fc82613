"""BaseModel (reference semseg/models/base.py:37-90): Swin-B / Swin-L variants only."""
import math

import torch
from torch import nn

from semseg.models.backbones import SwinTransformer  # noqa: F401  (resolved by name below)


def load_dualpath_model(model, model_file):
    raw = torch.load(model_file, map_location='cpu', weights_only=True) if isinstance(model_file, str) else model_file
    if 'model' in raw:
        raw = raw['model']
    keep = {k: v for k, v in raw.items() if ('patch_embed' in k) or ('block' in k) or ('norm' in k)}
    msg = model.load_state_dict(keep, strict=False)
    print(msg)


class BaseModel(nn.Module):
    def __init__(self, backbone: str = 'SwinTransformer-B', num_classes: int = 19,
                 modals: list = ['rgb', 'depth', 'event', 'lidar']) -> None:
        super().__init__()
        name, variant = backbone.split('-')
        cls = {'SwinTransformer': SwinTransformer}.get(name)
        if cls is None:
            raise ValueError('The backbone does not exist.')
        if variant == 'B':
            self.backbone = cls(with_cp=True) if 'event' in modals else cls()
        elif variant == 'L':
            self.backbone = cls(embed_dims=192, num_heads=(6, 12, 24, 48), with_cp=True)
        else:
            raise ValueError('The backbone does not exist.')
        self.modals = modals

    def _init_weights(self, m: nn.Module) -> None:
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Conv2d):
            fan_out = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
            m.weight.data.normal_(0, math.sqrt(2.0 / fan_out))
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, (nn.LayerNorm, nn.BatchNorm2d)):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)

    def init_pretrained(self, pretrained: str = None) -> None:
        if pretrained:
            if len(self.modals) > 1:
                load_dualpath_model(self.backbone, pretrained)
            else:
                ckpt = torch.load(pretrained, map_location='cpu', weights_only=True)
                ckpt = ckpt.get('state_dict', ckpt)
                ckpt = ckpt.get('model', ckpt)
                print(self.backbone.load_state_dict(ckpt, strict=False))
