"""Box conversions and (generalised) IoU (reference detrex/layers/box_ops.py:28-116; torchvision's
box_iou / generalized_box_iou formulas with the reference's 1e-6 guards)."""
import torch


def box_cxcywh_to_xyxy(bbox):
    cx, cy, w, h = bbox.unbind(-1)
    return torch.stack([cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h], dim=-1)


def box_xyxy_to_cxcywh(bbox):
    x0, y0, x1, y1 = bbox.unbind(-1)
    return torch.stack([(x0 + x1) / 2, (y0 + y1) / 2, x1 - x0, y1 - y0], dim=-1)


def _area(b):
    return (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])


def box_iou(boxes1, boxes2):
    """Pairwise IoU and union of two xyxy box sets: (N, M) each."""
    lt = torch.max(boxes1[:, None, :2], boxes2[:, :2])
    rb = torch.min(boxes1[:, None, 2:], boxes2[:, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[:, :, 0] * wh[:, :, 1]
    union = _area(boxes1)[:, None] + _area(boxes2) - inter
    return inter / (union + 1e-6), union


def generalized_box_iou(boxes1, boxes2):
    """Pairwise GIoU of xyxy boxes; degenerate boxes (x1 < x0) raise like the reference's assert."""
    if not bool((boxes1[:, 2:] >= boxes1[:, :2]).all()) or not bool((boxes2[:, 2:] >= boxes2[:, :2]).all()):
        raise AssertionError("generalized_box_iou: degenerate boxes")
    iou, union = box_iou(boxes1, boxes2)
    lt = torch.min(boxes1[:, None, :2], boxes2[:, :2])
    rb = torch.max(boxes1[:, None, 2:], boxes2[:, 2:])
    wh = (rb - lt).clamp(min=0)
    area = wh[:, :, 0] * wh[:, :, 1]
    return iou - (area - union) / (area + 1e-6)
