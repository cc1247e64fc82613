"""Datasets for the drivers (reference semseg/datasets/*).  The data pipeline is outside the
hot path; what is here is what train_mm.py / val_mm.py need: the NYU-Depth-v2
reader (reference layout: RGB/*.jpg, HHA/*.jpg, Label/*.png, train.txt / test.txt) and a
synthetic RGB-D set of the same shapes for offline runs."""
import os

import numpy as np
import torch
from torch.utils.data import Dataset

NYU_CLASSES = ['wall', 'floor', 'cabinet', 'bed', 'chair', 'sofa', 'table', 'door', 'window', 'bookshelf', 'picture',
               'counter', 'blinds', 'desk', 'shelves', 'curtain', 'dresser', 'pillow', 'mirror', 'floor mat',
               'clothes', 'ceiling', 'books', 'refridgerator', 'television', 'paper', 'towel', 'shower curtain',
               'box', 'whiteboard', 'person', 'night stand', 'toilet', 'sink', 'lamp', 'bathtub', 'bag',
               'otherstructure', 'otherfurniture', 'otherprop']


def _read(path):
    from PIL import Image
    a = np.asarray(Image.open(path))
    if a.ndim == 2:
        a = a[:, :, None]
    return torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1)


class NYU(Dataset):
    """num_classes: 40 (reference semseg/datasets/nyu.py)."""
    CLASSES = NYU_CLASSES
    PALETTE = None

    def __init__(self, root='data/NYUDepthv2', split='train', transform=None, modals=('img', 'depth'), case=None):
        super().__init__()
        assert split in ['train', 'val']
        self.root, self.transform, self.modals = root, transform, list(modals)
        self.n_classes = len(self.CLASSES)
        self.ignore_label = 255
        lst = os.path.join(root, 'train.txt' if split == 'train' else 'test.txt')
        with open(lst) as f:
            self.files = [ln.strip().split(' ')[0].split('/')[-1].split('.')[0] for ln in f if ln.strip()]
        if not self.files:
            raise Exception(f"No images found in {root}")

    def __len__(self):
        return len(self.files)

    def __getitem__(self, index):
        name = self.files[index]
        sample = {'img': _read(os.path.join(self.root, 'RGB', name + '.jpg'))[:3]}
        if 'depth' in self.modals:
            d = _read(os.path.join(self.root, 'HHA', name + '.jpg'))
            sample['depth'] = d[:3] if d.shape[0] >= 3 else d.repeat(3, 1, 1)
        label = _read(os.path.join(self.root, 'Label', name + '.png'))[:1].long()
        label[label == 255] = 0
        label -= 1  # 0 (unlabelled) -> -1 -> 255 after the uint8 wrap of the reference
        label[label < 0] = 255
        sample['mask'] = label
        if self.transform:
            sample = self.transform(sample)
        label = sample.pop('mask').squeeze(0).long()
        return [sample[k] for k in self.modals], label


class MFNet(Dataset):
    """MFNet RGB-T, num_classes 9 (reference semseg/datasets/mfnet.py: rgb/<name>.png,
    ther/<name>.png, labels/<name>.png; the file list is <split>.txt under ROOT)."""
    CLASSES = ['unlabeled', 'car', 'person', 'bike', 'curve', 'car_stop', 'guardrail', 'color_cone', 'bump']
    PALETTE = None

    def __init__(self, root='data/MFNet', split='train', transform=None, modals=('img', 'thermal'), case=None):
        super().__init__()
        assert split in ['train', 'val']
        self.root, self.transform, self.modals = root, transform, list(modals)
        self.n_classes = len(self.CLASSES)
        self.ignore_label = 255
        lst = os.path.join(root, f'{split}.txt')
        self.files = [ln.strip() for ln in open(lst)] if os.path.isfile(lst) else []
        if not self.files:
            raise Exception(f"No images found in {root}")

    def __len__(self):
        return len(self.files)

    def __getitem__(self, index):
        name = self.files[index]
        sample = {'img': _read(os.path.join(self.root, 'rgb', name + '.png'))[:3]}
        if 'thermal' in self.modals:
            t = _read(os.path.join(self.root, 'ther', name + '.png'))
            sample['thermal'] = t[:3] if t.shape[0] >= 3 else t[:1].repeat(3, 1, 1)
        sample['mask'] = _read(os.path.join(self.root, 'labels', name + '.png'))[:1].long()
        if self.transform:
            sample = self.transform(sample)
        label = sample.pop('mask').squeeze(0).long()
        return [sample[k] for k in self.modals], label


class Synthetic(Dataset):
    """Synthetic RGB-D batches with the NYU label space (the bench's data: RGB N(0,1) after
    Normalize, depth U[0,1), labels U{0..n-1} with ~10 % ignore)."""
    CLASSES = NYU_CLASSES

    def __init__(self, root=None, split='train', transform=None, modals=('img', 'depth'), case=None, length=16,
                 size=(512, 512), seed=3407):
        self.n_classes, self.ignore_label, self.modals = len(self.CLASSES), 255, list(modals)
        self.length, self.size, self.seed = length, tuple(size), seed + (0 if split == 'train' else 1)

    def __len__(self):
        return self.length

    def __getitem__(self, index):
        g = torch.Generator().manual_seed(self.seed * 100003 + index)
        H, W = self.size
        xs = [torch.randn(3, H, W, generator=g) if m == 'img' else torch.rand(3, H, W, generator=g)
              for m in self.modals]
        lbl = torch.randint(0, self.n_classes, (H, W), generator=g)
        lbl[torch.rand(H, W, generator=g) < 0.1] = 255
        return xs, lbl


__all__ = ['NYU', 'MFNet', 'Synthetic']
