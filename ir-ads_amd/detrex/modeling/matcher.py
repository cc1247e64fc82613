"""Hungarian matcher (reference detrex/modeling/matcher/matcher.py:36-150): focal-loss class cost,
L1 box cost and GIoU cost, solved per image with scipy's linear_sum_assignment on the host."""
import torch
import torch.nn as nn
from scipy.optimize import linear_sum_assignment

from detrex.layers.box_ops import box_cxcywh_to_xyxy, generalized_box_iou


class HungarianMatcher(nn.Module):
    def __init__(self, cost_class=1.0, cost_bbox=1.0, cost_giou=1.0, cost_class_type="focal_loss_cost",
                 alpha=0.25, gamma=2.0):
        super().__init__()
        assert cost_class != 0 or cost_bbox != 0 or cost_giou != 0, "all costs cant be 0"
        assert cost_class_type in {"ce_cost", "focal_loss_cost"}
        self.cost_class, self.cost_bbox, self.cost_giou = cost_class, cost_bbox, cost_giou
        self.cost_class_type, self.alpha, self.gamma = cost_class_type, alpha, gamma

    @torch.no_grad()
    def forward(self, outputs, targets):
        """[(query indices, target indices)] per image, both int64 on the CPU (as the reference)."""
        bs, nq = outputs["pred_logits"].shape[:2]
        logits = outputs["pred_logits"].flatten(0, 1)
        out_bbox = outputs["pred_boxes"].flatten(0, 1)
        tgt_ids = torch.cat([v["labels"] for v in targets])
        tgt_bbox = torch.cat([v["boxes"] for v in targets])
        if self.cost_class_type == "ce_cost":
            cost_class = -logits.softmax(-1)[:, tgt_ids]
        else:
            p = logits.sigmoid()
            neg = (1 - self.alpha) * (p ** self.gamma) * (-(1 - p + 1e-8).log())
            pos = self.alpha * ((1 - p) ** self.gamma) * (-(p + 1e-8).log())
            cost_class = pos[:, tgt_ids] - neg[:, tgt_ids]
        cost_bbox = torch.cdist(out_bbox, tgt_bbox, p=1)
        cost_giou = -generalized_box_iou(box_cxcywh_to_xyxy(out_bbox), box_cxcywh_to_xyxy(tgt_bbox))
        C = (self.cost_bbox * cost_bbox + self.cost_class * cost_class + self.cost_giou * cost_giou)
        C = C.view(bs, nq, -1).cpu()
        sizes = [len(v["boxes"]) for v in targets]
        idx = [linear_sum_assignment(c[i]) for i, c in enumerate(C.split(sizes, -1))]
        return [(torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64)) for i, j in idx]
