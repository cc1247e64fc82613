"""CMNeXt with the two-stream Swin backbone (reference semseg/models/cmnext.py:11-36)."""
import torch

from irads import amp_cache, ops
from semseg.models.base import BaseModel
from semseg.models.heads import SegFormerHead


class CMNeXt(BaseModel):
    def __init__(self, backbone: str = 'SwinTransformer-B', num_classes: int = 25,
                 modals: list = ['img', 'depth', 'event', 'lidar']) -> None:
        super().__init__(backbone, num_classes, modals)
        if backbone == 'SwinTransformer-B':
            channels = [128, 256, 512, 1024]
        elif backbone == 'SwinTransformer-L':
            channels = [192, 384, 768, 1536]
        else:
            raise ValueError('The backbone does not exist.')
        self.decode_head = SegFormerHead(channels, 512, num_classes)
        self.decode_head_rgb = SegFormerHead(channels, 256, num_classes)
        self.decode_head_dte = SegFormerHead(channels, 256, num_classes)
        self.apply(self._init_weights)

    def forward(self, x: list):
        if (self.training and x[0].is_cuda and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            # all trainable weights cast to bf16 in one pass (irads/amp_cache.py)
            amp_cache.refresh([p for p in self.parameters() if p.requires_grad])
        y, y_rgb, y_dte = self.backbone(x)
        size = x[0].shape[2:]
        # F.interpolate(..., mode='bilinear', align_corners=False) on the HIP resize kernels
        y = ops.resize(self.decode_head(y), size)
        y_rgb = ops.resize(self.decode_head_rgb(y_rgb), size)
        y_dte = ops.resize(self.decode_head_dte(y_dte), size)
        return y, y_rgb, y_dte

    def init_pretrained(self, pretrained: str = None) -> None:
        self.backbone.init_weights()
