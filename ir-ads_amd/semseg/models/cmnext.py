"""CMNeXt with the two-stream Swin backbone (reference semseg/models/cmnext.py:11-36)."""
import torch

from irads import amp_cache, ops
from semseg.models.base import BaseModel
from semseg.models.heads import SegFormerHead


class CMNeXt(BaseModel):
    """sb: None (the reference model) or a dict enabling the build-defined Schrödinger-bridge hook
    (DESIGN.md §SB hook; the reference's modules/sb.py has no caller):
    {'weight': 0.01, 'n_potentials': 10, 'epsilon': 0.1}.  With it, a LightSB(dim=512) is fitted
    on the fused head's 512-d per-pixel feature (cmnext.py:20, 1/4 resolution) by LightSB's own
    objective with x0 = x1 = those features (a self-bridge: its potential is a density model of
    the features), through sb_loss(); sb_anomaly_map() = -log v of the last forward's features."""

    def __init__(self, backbone: str = 'SwinTransformer-B', num_classes: int = 25,
                 modals: list = ['img', 'depth', 'event', 'lidar'], sb: dict = None) -> None:
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
        self.sb_cfg = dict(sb) if sb else None
        if self.sb_cfg:
            from modules.sb import LightSB
            self.sb = LightSB(dim=512, n_potentials=int(self.sb_cfg.get('n_potentials', 10)),
                              epsilon=float(self.sb_cfg.get('epsilon', 0.1)))
            self.decode_head.keep_feature = True

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

    def _sb_rows(self):
        f = self.decode_head.feature  # (B, h*w, 512) tokens of the last forward
        return f.reshape(-1, f.shape[-1]).detach().float()

    def sb_loss(self):
        """weight * (E[log C(x0)] - E[log v(x1)]), x0 = x1 = the fused head's feature rows
        (LightSB's training objective; the features are detached: the hook trains the bridge,
        not the backbone)."""
        x = self._sb_rows()
        return float(self.sb_cfg.get('weight', 0.01)) * (self.sb.get_log_C(x).mean()
                                                          - self.sb.get_log_potential(x).mean())

    @torch.no_grad()
    def sb_anomaly_map(self):
        """-log v(feature) per pixel of the last forward, (B, h, w) at the head's 1/4 resolution."""
        f = self.decode_head.feature
        B = f.shape[0]
        h, w = self.decode_head.feature_hw
        return -self.sb.get_log_potential(self._sb_rows()).view(B, h, w)

    def init_pretrained(self, pretrained: str = None) -> None:
        self.backbone.init_weights()
