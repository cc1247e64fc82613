"""Losses (reference semseg/losses.py) and the MMST objective of train_mm.py:137-148."""
import torch
from torch import nn, Tensor
from torch.nn import functional as F

from irads import ops


class CrossEntropy(nn.Module):
    def __init__(self, ignore_label: int = 255, weight: Tensor = None, aux_weights: list = [1, 0.4, 0.4]) -> None:
        super().__init__()
        self.aux_weights = aux_weights
        self.criterion = nn.CrossEntropyLoss(weight=weight, ignore_index=ignore_label)

    def _forward(self, preds: Tensor, labels: Tensor) -> Tensor:
        # nn.CrossEntropyLoss semantics (mean over non-ignored pixels, optional class
        # weights) on the fused HIP kernel; the criterion module keeps weight/ignore_index
        return ops.cross_entropy(preds, labels, self.criterion.ignore_index, self.criterion.weight)

    def forward(self, preds, labels: Tensor) -> Tensor:
        if isinstance(preds, tuple):
            return sum(w * self._forward(p, labels) for p, w in zip(preds, self.aux_weights))
        return self._forward(preds, labels)


class OhemCrossEntropy(nn.Module):
    def __init__(self, ignore_label: int = 255, weight: Tensor = None, thresh: float = 0.7,
                 aux_weights: list = [1, 1]) -> None:
        super().__init__()
        self.ignore_label = ignore_label
        self.aux_weights = aux_weights
        self.thresh = -torch.log(torch.tensor(thresh, dtype=torch.float))
        self.criterion = nn.CrossEntropyLoss(weight=weight, ignore_index=ignore_label, reduction='none')

    def _forward(self, preds: Tensor, labels: Tensor) -> Tensor:
        n_min = labels[labels != self.ignore_label].numel() // 16
        loss = self.criterion(preds, labels).view(-1)
        hard = loss[loss > self.thresh]
        if hard.numel() < n_min:
            hard, _ = loss.topk(n_min)
        return torch.mean(hard)

    def forward(self, preds, labels: Tensor) -> Tensor:
        if isinstance(preds, tuple):
            return sum(w * self._forward(p, labels) for p, w in zip(preds, self.aux_weights))
        return self._forward(preds, labels)


class Dice(nn.Module):
    def __init__(self, delta: float = 0.5, aux_weights: list = [1, 0.4, 0.4]):
        super().__init__()
        self.delta = delta
        self.aux_weights = aux_weights

    def _forward(self, preds: Tensor, labels: Tensor) -> Tensor:
        n = preds.shape[1]
        labels = F.one_hot(labels, n).permute(0, 3, 1, 2)
        tp = torch.sum(labels * preds, dim=(2, 3))
        fn = torch.sum(labels * (1 - preds), dim=(2, 3))
        fp = torch.sum((1 - labels) * preds, dim=(2, 3))
        dice = (tp + 1e-6) / (tp + self.delta * fn + (1 - self.delta) * fp + 1e-6)
        return (torch.sum(1 - dice, dim=-1) / n).mean()

    def forward(self, preds, targets: Tensor) -> Tensor:
        if isinstance(preds, tuple):
            return sum(w * self._forward(p, targets) for p, w in zip(preds, self.aux_weights))
        return self._forward(preds, targets)


__all__ = ['CrossEntropy', 'OhemCrossEntropy', 'Dice']


def get_loss(loss_fn_name: str = 'CrossEntropy', ignore_label: int = 255, cls_weights: Tensor = None):
    assert loss_fn_name in __all__, f"Unavailable loss function name >> {loss_fn_name}.\nAvailable loss functions: {__all__}"
    if loss_fn_name == 'Dice':
        return Dice()
    return {'CrossEntropy': CrossEntropy, 'OhemCrossEntropy': OhemCrossEntropy}[loss_fn_name](ignore_label, cls_weights)


def mmst_loss(loss_fn, logits, logits_rgb, logits_dte, lbl, ignore_label=255):
    """train_mm.py:137-148: pixels the fused head gets wrong are ignored (255) for the
    two auxiliary modality heads, each weighted 0.01.  With CrossEntropy the MMST target
    (label where argmax(softmax(logits)) == label) comes out of the fused loss pass of the
    main head; argmax of the softmax equals the first argmax of the logits, since
    distinct bf16/fp32 logits give distinct fp32 probabilities."""
    if isinstance(loss_fn, CrossEntropy) and not isinstance(logits, tuple):
        crit = loss_fn.criterion
        loss1, mask_lbl = ops.cross_entropy(logits, lbl, crit.ignore_index, crit.weight, return_match=True)
        return loss1 + 0.01 * loss_fn(logits_rgb, mask_lbl) + 0.01 * loss_fn(logits_dte, mask_lbl)
    with torch.no_grad():
        pred = logits.softmax(dim=1).argmax(dim=1)
        mask_lbl = torch.where(pred == lbl, lbl, torch.full_like(lbl, ignore_label))
    return loss_fn(logits, lbl) + 0.01 * loss_fn(logits_rgb, mask_lbl) + 0.01 * loss_fn(logits_dte, mask_lbl)
