"""Segmentation metrics (reference semseg/metrics.py:45-96), accumulated on the GPU.

The reference keeps per-class tp/fp/fn as Python ints and pays 3 x n_classes `.item()`
host synchronisations per batch (metrics.py:64-69).  Here `update` is one kernel
(irads_confusion_update: arg-max + confusion matrix in one pass over the scores, no host
round trip) and the tp/fp/fn lists are read once, when a result is asked for.  The
public interface and the arithmetic of compute_iou are the reference's: per class
tp / max(tp + fp + fn, 1e-8) as Python floats, mIoU = round(mean * 100, 2), the per-class
list returned unrounded (the reference's rounding loop does not modify it).
"""
import numpy as np
import torch

from irads import ops


class Metrics:
    def __init__(self, num_classes: int, ignore_label: int, device) -> None:
        self.n_classes = num_classes
        self.ignore_idx = ignore_label
        self.device = torch.device(device)
        self.hist = torch.zeros(((num_classes + 1) * num_classes,), dtype=torch.int64, device=self.device)

    @torch.no_grad()
    def update(self, pred, gt) -> None:
        """pred (B, C, H, W) scores (logits or probabilities), gt (B, H, W)."""
        ops.confusion_update(pred, gt, self.ignore_idx, self.hist)

    def reset(self) -> None:
        self.hist.zero_()

    def _counts(self):
        C = self.n_classes
        h = self.hist.view(C + 1, C).cpu()
        diag = torch.diagonal(h[:C])
        tp = diag.tolist()
        fp = (h.sum(0) - diag).tolist()
        fn = (h[:C].sum(1) - diag).tolist()
        return tp, fp, fn

    @property
    def tp(self):
        return self._counts()[0]

    @property
    def fp(self):
        return self._counts()[1]

    @property
    def fn(self):
        return self._counts()[2]

    def compute_iou(self, verbose=True):
        tp, fp, fn = self._counts()
        jac = [float(tp[i]) / max(float(tp[i] + fp[i] + fn[i]), 1e-8) for i in range(self.n_classes)]
        return jac, round(float(np.mean(jac)) * 100, 2)  # a Python float: checkpoints stay weights_only-loadable

    def compute_f1(self):
        tp, fp, fn = self._counts()
        f1 = [2.0 * tp[i] / max(float(2 * tp[i] + fp[i] + fn[i]), 1e-8) for i in range(self.n_classes)]
        return [round(v * 100, 2) for v in f1], round(float(np.mean(f1)) * 100, 2)

    def compute_pixel_acc(self):
        tp, _, fn = self._counts()
        acc = [float(tp[i]) / max(float(tp[i] + fn[i]), 1e-8) for i in range(self.n_classes)]
        return [round(v * 100, 2) for v in acc], round(float(np.mean(acc)) * 100, 2)
