"""CMNeXt with the two-stream Swin backbone (reference semseg/models/cmnext.py:11-36)."""
from torch.nn import functional as F

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
        y, y_rgb, y_dte = self.backbone(x)
        size = x[0].shape[2:]
        y = F.interpolate(self.decode_head(y), size=size, mode='bilinear', align_corners=False)
        y_rgb = F.interpolate(self.decode_head_rgb(y_rgb), size=size, mode='bilinear', align_corners=False)
        y_dte = F.interpolate(self.decode_head_dte(y_dte), size=size, mode='bilinear', align_corners=False)
        return y, y_rgb, y_dte

    def init_pretrained(self, pretrained: str = None) -> None:
        self.backbone.init_weights()
