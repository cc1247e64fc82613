"""Multimodal augmentations (reference semseg/augmentations_mm.py), CPU loader side.
Outside the hot path; implements the transforms the NYU configs use: horizontal flip,
random resized crop (scale 0.5-2.0, mask filled with the ignore label), Resize to a multiple
of 32 (val) and Normalize (ImageNet statistics for 'img', /255 for the other modalities)."""
import math
import random

import torch
import torch.nn.functional as F


def _resize(t, size, nearest):
    x = t.unsqueeze(0).float()
    if nearest:
        return F.interpolate(x, size=size, mode='nearest')[0].to(t.dtype)
    return F.interpolate(x, size=size, mode='bilinear', align_corners=False, antialias=False)[0]


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, sample):
        for t in self.transforms:
            sample = t(sample)
        return sample


class Normalize:
    def __init__(self, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
        self.mean = torch.tensor(mean).view(3, 1, 1)
        self.std = torch.tensor(std).view(3, 1, 1)

    def __call__(self, sample):
        for k, v in sample.items():
            if k == 'mask':
                continue
            v = v.float() / 255
            sample[k] = (v - self.mean) / self.std if k == 'img' else v
        return sample


class RandomHorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, sample):
        if random.random() < self.p:
            return {k: v.flip(-1) for k, v in sample.items()}
        return sample


class Resize:
    def __init__(self, size):
        self.size = size

    def __call__(self, sample):
        H, W = sample['img'].shape[1:]
        s = self.size[0] / min(H, W)
        nH, nW = round(H * s), round(W * s)
        aH, aW = int(math.ceil(nH / 32)) * 32, int(math.ceil(nW / 32)) * 32
        for k, v in sample.items():
            sample[k] = _resize(_resize(v, (nH, nW), k == 'mask'), (aH, aW), k == 'mask')
        return sample


class RandomResizedCrop:
    def __init__(self, size, scale=(0.5, 2.0), seg_fill=0):
        self.size, self.scale, self.seg_fill = size, scale, seg_fill

    def __call__(self, sample):
        H, W = sample['img'].shape[1:]
        tH, tW = self.size
        ratio = random.random() * (self.scale[1] - self.scale[0]) + self.scale[0]
        s = int(tH * ratio) / max(H, W)
        nH, nW = max(1, int(H * s + 0.5)), max(1, int(W * s + 0.5))
        for k, v in sample.items():
            sample[k] = _resize(v, (nH, nW), k == 'mask')
        mh, mw = max(nH - tH, 0), max(nW - tW, 0)
        y0, x0 = random.randint(0, mh), random.randint(0, mw)
        for k, v in sample.items():
            v = v[:, y0:y0 + tH, x0:x0 + tW]
            if v.shape[1:] != (tH, tW):
                pad = (0, tW - v.shape[2], 0, tH - v.shape[1])
                v = F.pad(v.float(), pad, value=self.seg_fill if k == 'mask' else 0).to(v.dtype)
            sample[k] = v
        return sample


def get_train_augmentation(size, seg_fill=0):
    return Compose([RandomHorizontalFlip(p=0.5), RandomResizedCrop(size, scale=(0.5, 2.0), seg_fill=seg_fill),
                    Normalize((0.485, 0.456, 0.406), (0.229, 0.224, 0.225))])


def get_val_augmentation(size):
    return Compose([Resize(size), Normalize((0.485, 0.456, 0.406), (0.229, 0.224, 0.225))])
