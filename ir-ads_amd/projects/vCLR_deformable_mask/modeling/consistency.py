"""Siamese consistency loss of the vCLR detector (reference
projects/vCLR_deformable_mask/modeling/ConsisCriterion.py:26-106, built at
configs/models/dino_r50.py:110-130 with its own Hungarian matcher: class 2 / L1 5 / GIoU 2, focal).

The student's last-layer queries and the EMA teacher's (DINO.infer_results, on the weak view) are
each Hungarian-matched to the ground truth; for every ground-truth box the two matched query
features are compared: loss_sim = -mean cosine similarity (the teacher's side detached).  The
matches are ordered by ground-truth index on both sides, so pair k is "the queries both views
assigned to box k".  ``num_boxes`` is computed and all-reduced as the reference does (a collective
every rank joins), although the loss does not use it."""
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


def _by_target(indices):
    """(query index, target index) pairs of each image reordered by target index."""
    out = []
    for q, t in indices:
        order = torch.argsort(t)
        out.append((q[order], t[order]))
    return out


def _flat_index(indices):
    batch = torch.cat([torch.full_like(q, b) for b, (q, _) in enumerate(indices)])
    return batch, torch.cat([q for q, _ in indices])


class ConsisCriterion(nn.Module):
    def __init__(self, matcher, weight_dict):
        super().__init__()
        self.matcher = matcher
        self.weight_dict = weight_dict

    def forward(self, outputs, siamese_outputs, targets, dn_meta=None):
        student = _by_target(self.matcher({k: v for k, v in outputs.items() if k != "aux_outputs"}, targets))
        teacher = _by_target(self.matcher(siamese_outputs, targets))
        dev = outputs["pred_logits"].device
        num_boxes = torch.as_tensor([float(sum(len(t["labels"]) for t in targets))], device=dev)
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(num_boxes)
        src = outputs["pred_queries"][_flat_index(student)]
        tgt = siamese_outputs["pred_query"][_flat_index(teacher)]
        return {"loss_sim": -F.cosine_similarity(src, tgt.detach(), dim=1).mean()}
