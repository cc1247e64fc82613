"""vCLR DINO criterion (reference projects/vCLR_deformable_mask/modeling/two_stage_criterion.py:32-424
and dn_criterion.py:20-137 on detrex/modeling/criterion/criterion.py's SetCriterion): Hungarian
matching of the last layer, every auxiliary layer and the two-stage encoder proposals; sigmoid
focal class loss, L1 + GIoU box losses, point-sampled mask losses (sigmoid BCE + dice at
uncertainty-weighted points: detectron2 point_rend's get_uncertain_point_coords_with_randomness /
point_sample, restated in ``point_sample`` / ``uncertain_points``), the zero-weighted ROI term, and
the contrastive-denoising losses of the known queries.  ``num_boxes`` is all-reduced over the
ranks (dn_criterion.py:43-46) when a process group is up.

Random draws go through ``self.rng`` (``torch`` by default); the parity test replays the
reference's recorded draws through it."""
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from detrex.layers.box_ops import box_cxcywh_to_xyxy, generalized_box_iou


def sigmoid_focal_loss(inputs, targets, num_boxes, alpha=0.25, gamma=2.0):
    prob = inputs.sigmoid()
    ce = F.binary_cross_entropy_with_logits(inputs, targets, reduction="none")
    p_t = prob * targets + (1 - prob) * (1 - targets)
    loss = ce * ((1 - p_t) ** gamma)
    if alpha >= 0:
        loss = (alpha * targets + (1 - alpha) * (1 - targets)) * loss
    return loss.mean(1).sum() / num_boxes


def dice_loss(inputs, targets, num_masks):
    inputs = inputs.sigmoid().flatten(1)
    num = 2 * (inputs * targets).sum(-1)
    den = inputs.sum(-1) + targets.sum(-1)
    return (1 - (num + 1) / (den + 1)).sum() / num_masks


def sigmoid_ce_loss(inputs, targets, num_masks):
    return F.binary_cross_entropy_with_logits(inputs, targets, reduction="none").mean(1).sum() / num_masks


def point_sample(inp, coords, **kwargs):
    """grid_sample at normalised [0, 1] point coordinates (N, P, 2) -> (N, C, P)."""
    out = F.grid_sample(inp, 2.0 * coords.unsqueeze(2) - 1.0, **kwargs)
    return out.squeeze(3)


def uncertain_points(logits, num_points, oversample_ratio, importance_ratio, rng=torch):
    """Oversample uniformly, keep the importance_ratio most uncertain (|logit| smallest), fill the
    rest uniformly (point_rend's get_uncertain_point_coords_with_randomness)."""
    n = logits.shape[0]
    n_sampled = int(num_points * oversample_ratio)
    coords = rng.rand(n, n_sampled, 2, device=logits.device, dtype=logits.dtype)
    unc = -point_sample(logits, coords, align_corners=False).abs()
    n_unc = int(importance_ratio * num_points)
    n_rand = num_points - n_unc
    idx = torch.topk(unc[:, 0, :], k=n_unc, dim=1)[1]
    idx = idx + n_sampled * torch.arange(n, dtype=torch.long, device=logits.device)[:, None]
    coords = coords.view(-1, 2)[idx.view(-1), :].view(n, n_unc, 2)
    if n_rand > 0:
        coords = torch.cat([coords, rng.rand(n, n_rand, 2, device=logits.device, dtype=logits.dtype)], dim=1)
    return coords


def _padded_masks(masks):
    """Stack per-image (n_i, H, W) masks into (B, max n, H, W) zero-padded (misc.py:48-73)."""
    n = max(m.shape[0] for m in masks)
    H = max(m.shape[1] for m in masks)
    W = max(m.shape[2] for m in masks)
    out = masks[0].new_zeros((len(masks), n, H, W))
    for o, m in zip(out, masks):
        o[:m.shape[0], :m.shape[1], :m.shape[2]].copy_(m)
    return out


def _num_boxes(targets, device):
    n = torch.as_tensor([float(sum(len(t["labels"]) for t in targets))], device=device)
    world = 1
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(n)
        world = dist.get_world_size()
    return torch.clamp(n / world, min=1).item()


class DINOCriterion(nn.Module):
    def __init__(self, num_classes, matcher, weight_dict, losses=("class", "boxes", "masks"), eos_coef=None,
                 loss_class_type="focal_loss", alpha=0.25, gamma=2.0, two_stage_binary_cls=False):
        super().__init__()
        assert loss_class_type == "focal_loss", "the vCLR config trains with focal_loss"
        self.num_classes, self.matcher, self.weight_dict = num_classes, matcher, weight_dict
        self.losses, self.alpha, self.gamma = list(losses), alpha, gamma
        self.two_stage_binary_cls = two_stage_binary_cls
        self.num_points, self.oversample_ratio, self.importance_sample_ratio = 12544, 3.0, 0.75
        self.rng = torch

    # ---------------------------------------------------------------- indices
    @staticmethod
    def _src_idx(indices):
        return (torch.cat([torch.full_like(s, i) for i, (s, _) in enumerate(indices)]),
                torch.cat([s for s, _ in indices]))

    @staticmethod
    def _tgt_idx(indices):
        return (torch.cat([torch.full_like(t, i) for i, (_, t) in enumerate(indices)]),
                torch.cat([t for _, t in indices]))

    # ---------------------------------------------------------------- losses
    def loss_labels(self, outputs, targets, indices, num_boxes):
        logits = outputs["pred_logits"]
        idx = self._src_idx(indices)
        tc_o = torch.cat([t["labels"][J] for t, (_, J) in zip(targets, indices)])
        tc = torch.full(logits.shape[:2], self.num_classes, dtype=torch.int64, device=logits.device)
        tc[idx] = tc_o.to(logits.device)
        onehot = torch.zeros((logits.shape[0], logits.shape[1], logits.shape[2] + 1), dtype=logits.dtype,
                             device=logits.device)
        onehot.scatter_(2, tc.unsqueeze(-1), 1)
        loss = sigmoid_focal_loss(logits, onehot[:, :, :-1], num_boxes, self.alpha, self.gamma) * logits.shape[1]
        return {"loss_class": loss}

    def loss_boxes(self, outputs, targets, indices, num_boxes):
        idx = self._src_idx(indices)
        src = outputs["pred_boxes"][idx]
        tgt = torch.cat([t["boxes"][i] for t, (_, i) in zip(targets, indices)], dim=0)
        losses = {"loss_bbox": F.l1_loss(src, tgt, reduction="none").sum() / num_boxes}
        if "pred_rois" in outputs:  # the ROI-feature term is weighted by zero (two_stage_criterion.py:344-350)
            losses["loss_roi"] = outputs["pred_rois"].mean() * 0.
        else:
            losses["loss_roi"] = torch.zeros(1, device=src.device)
        giou = 1 - torch.diag(generalized_box_iou(box_cxcywh_to_xyxy(src), box_cxcywh_to_xyxy(tgt)))
        losses["loss_giou"] = giou.sum() / num_boxes
        return losses

    def loss_masks(self, outputs, targets, indices, num_masks):
        src = outputs["pred_masks"][self._src_idx(indices)][:, None]
        tmasks = _padded_masks([t["masks"] for t in targets]).to(src)
        tgt = tmasks[self._tgt_idx(indices)][:, None]
        with torch.no_grad():
            coords = uncertain_points(src, self.num_points, self.oversample_ratio, self.importance_sample_ratio,
                                      self.rng)
            labels = point_sample(tgt, coords, align_corners=False).squeeze(1)
        logits = point_sample(src, coords, align_corners=False).squeeze(1)
        return {"loss_mask": sigmoid_ce_loss(logits, labels, num_masks),
                "loss_dice": dice_loss(logits, labels, num_masks)}

    def get_loss(self, loss, outputs, targets, indices, num_boxes):
        return {"class": self.loss_labels, "boxes": self.loss_boxes, "masks": self.loss_masks}[loss](
            outputs, targets, indices, num_boxes)

    # ---------------------------------------------------------------- forward
    def forward(self, outputs, targets, dn_metas=None):
        dev = outputs["pred_logits"].device
        num_boxes = _num_boxes(targets, dev)
        losses = {}
        main = {k: v for k, v in outputs.items() if k != "aux_outputs"}
        indices = self.matcher(main, targets)
        for loss in self.losses:
            losses.update(self.get_loss(loss, outputs, targets, indices, num_boxes))
        for i, aux in enumerate(outputs.get("aux_outputs", [])):
            indices = self.matcher(aux, targets)
            for loss in self.losses:
                losses.update({k + f"_{i}": v for k, v in self.get_loss(loss, aux, targets, indices,
                                                                           num_boxes).items()})
        if "enc_outputs" in outputs:
            enc = outputs["enc_outputs"]
            if self.two_stage_binary_cls:
                for t in targets:
                    t["labels"] = torch.zeros_like(t["labels"])
            indices = self.matcher(enc, targets)
            for loss in self.losses:
                losses.update({k + "_enc": v for k, v in self.get_loss(loss, enc, targets, indices,
                                                                        num_boxes).items()})
        # contrastive denoising (dn_criterion.py:37-137): num_boxes is all-reduced again there
        num_boxes = _num_boxes(targets, dev)
        aux_num = len(outputs.get("aux_outputs", []))
        losses.update(self.compute_dn_loss(dn_metas, targets, aux_num, num_boxes, dev))
        return losses

    def compute_dn_loss(self, dn_metas, targets, aux_num, num_boxes, dev):
        losses = {}
        names = ("loss_bbox", "loss_giou", "loss_class", "loss_roi", "loss_mask", "loss_dice")
        have = bool(dn_metas) and "output_known_lbs_bboxes" in dn_metas
        if have:
            known, dn_num, single = dn_metas["output_known_lbs_bboxes"], dn_metas["dn_num"], dn_metas["single_padding"]
            dn_idx = []
            for t in targets:
                if len(t["labels"]) > 0:
                    tt = torch.arange(0, len(t["labels"])).long().to(dev).unsqueeze(0).repeat(dn_num, 1)
                    tgt_idx = tt.flatten()
                    out_idx = ((torch.tensor(range(dn_num)) * single).long().to(dev).unsqueeze(1) + tt).flatten()
                else:
                    out_idx = tgt_idx = torch.tensor([]).long().to(dev)
                dn_idx.append((out_idx, tgt_idx))
            l_dict = {}
            for loss in ("class", "boxes", "masks"):
                l_dict.update(self.get_loss(loss, known, targets, dn_idx, num_boxes * dn_num))
            losses.update({k + "_dn": v for k, v in l_dict.items()})
        else:
            losses.update({k + "_dn": torch.as_tensor(0.0, device=dev) for k in names})
        for i in range(aux_num):
            if have:
                l_dict = {}
                for loss in ("class", "boxes", "masks"):
                    l_dict.update(self.get_loss(loss, known["aux_outputs"][i], targets, dn_idx, num_boxes * dn_num))
                losses.update({k + f"_dn_{i}": v for k, v in l_dict.items()})
            else:  # the reference's key spelling for this branch (dn_criterion.py:128-135)
                losses.update({k + f"_dn_{i}": torch.as_tensor(0.0, device=dev) for k in names})
        return losses
