"""Seeded inputs and the reduced configuration of the vCLR DINO detector training-step case
(TEST INFRASTRUCTURE): shared by the fixture generator (oracle/gen_golden.py gen_dino_detector,
reference side) and tests/test_gpu_dino_detector.py (product side).

Reduced from configs/models/dino_r50.py: 2 + 2 transformer layers (6 + 6), 30 two-stage queries
(900), 10 denoising groups' budget (100), 112 mask points per box (12 544); everything else as
configured (ResNet-50, ChannelMapper, 80 classes, label noise 0.5, box noise 1.0, loss weights).
Two images of different sizes (the second padded), 3 and 2 ground-truth boxes with box masks.

Random draws (denoising label / box noise, mask point sampling) come from a RecordingRNG on the
reference side; the fixture stores them and the product replays them (ReplayRNG), so both sides
use the same noise."""
import numpy as np
import torch

from fill import seeded

DET_CFG = dict(num_classes=80, num_queries=30, enc_layers=2, dec_layers=2, dn_number=10, label_noise_ratio=0.5,
               box_noise_scale=1.0)
DET_NUM_POINTS = 112
DET_IMAGE_SIZES = [(128, 160), (112, 144)]
DET_N_GT = [3, 2]
DET_FILL_SEED = 71
_RAND, _RANDINT = torch.rand, torch.randint  # the generator's own draws (torch.rand may be patched)


def det_inputs():
    """[(image (3, H, W) float in [0, 255), boxes xyxy pixels (n, 4), classes (n,), masks (n, H, W) bool)]."""
    out = []
    for i, ((H, W), n) in enumerate(zip(DET_IMAGE_SIZES, DET_N_GT)):
        img = np.floor(seeded((3, H, W), 300 + i, "uniform") * 255.0)
        u = seeded((n, 4), 310 + i, "uniform")
        x0 = np.floor(u[:, 0] * 0.6 * W)
        y0 = np.floor(u[:, 1] * 0.6 * H)
        x1 = np.minimum(W, x0 + 12 + np.floor(u[:, 2] * 0.4 * W))
        y1 = np.minimum(H, y0 + 12 + np.floor(u[:, 3] * 0.4 * H))
        boxes = np.stack([x0, y0, x1, y1], 1)
        cls = (seeded((n,), 320 + i, "uniform") * 80).astype(np.int64)
        masks = np.zeros((n, H, W), dtype=bool)
        for k in range(n):
            masks[k, int(y0[k]):int(y1[k]), int(x0[k]):int(x1[k])] = True
        out.append((img, boxes, cls, masks))
    return out


class RecordingRNG:
    """torch.rand / rand_like / randint_like from a seeded CPU generator; every draw is kept."""

    def __init__(self, seed):
        self.g = torch.Generator().manual_seed(seed)
        self.draws = []

    def _keep(self, t):
        self.draws.append(t.clone())
        return t

    def rand(self, *size, device=None, dtype=None, **kw):
        if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
            size = tuple(size[0])
        t = self._keep(_RAND(size, generator=self.g, dtype=torch.float64))
        return t.to(device=device, dtype=dtype or torch.get_default_dtype())

    def rand_like(self, x, **kw):
        return self._keep(_RAND(tuple(x.shape), generator=self.g, dtype=torch.float64)).to(x)

    def randint_like(self, x, low=0, high=None, dtype=None, **kw):
        if high is None:
            low, high = 0, low
        t = self._keep(_RANDINT(low, high, tuple(x.shape), generator=self.g, dtype=torch.int64))
        return t.to(device=x.device, dtype=dtype or x.dtype)

    def randint(self, low=0, high=None, size=None, dtype=None, device=None, **kw):
        if high is None:
            low, high = 0, low
        t = self._keep(_RANDINT(low, high, tuple(size), generator=self.g, dtype=torch.int64))
        return t.to(device=device, dtype=dtype or torch.int64)


class RecordingPyRandom:
    """random.uniform / randint / random from a seeded random.Random; every result is kept."""

    def __init__(self, seed):
        import random
        self.r = random.Random(seed)
        self.draws = []

    def _keep(self, v):
        self.draws.append(float(v))
        return v

    def uniform(self, a, b):
        return self._keep(self.r.uniform(a, b))

    def randint(self, a, b):
        return self._keep(self.r.randint(a, b))

    def random(self):
        return self._keep(self.r.random())


class ReplayPyRandom:
    """The recorded Python-random results, in order (randint's as ints)."""

    def __init__(self, draws):
        self.draws, self.i = [float(d) for d in draws], 0

    def _next(self):
        v = self.draws[self.i]
        self.i += 1
        return v

    def uniform(self, a, b):
        return self._next()

    def randint(self, a, b):
        v = self._next()
        assert v == int(v) and a <= v <= b, (v, a, b)
        return int(v)

    def random(self):
        return self._next()


class ReplayRNG:
    """The recorded draws, in order, on the caller's device and dtype."""

    def __init__(self, draws):
        self.draws, self.i = list(draws), 0

    def _next(self, shape):
        t = torch.as_tensor(self.draws[self.i])
        self.i += 1
        assert tuple(t.shape) == tuple(shape), (self.i - 1, tuple(t.shape), tuple(shape))
        return t

    def rand(self, *size, device=None, dtype=None, **kw):
        if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
            size = tuple(size[0])
        return self._next(size).to(device=device, dtype=dtype or torch.get_default_dtype())

    def rand_like(self, x, **kw):
        return self._next(x.shape).to(x)

    def randint_like(self, x, low=0, high=None, dtype=None, **kw):
        return self._next(x.shape).to(device=x.device, dtype=dtype or x.dtype)

    def randint(self, low=0, high=None, size=None, dtype=None, device=None, **kw):
        return self._next(tuple(size)).to(device=device, dtype=dtype or torch.int64)


TRAIN_PY_SEED = 0  # python-random seed of the training-forward case (its grayscale draw is > 0.5)
EMA_MIX = (0.9, 0.1, 1)  # teacher = 0.9 * the model's fill + 0.1 * the fill at DET_FILL_SEED + 1


def det_train_inputs():
    """det_inputs() plus each image's weak view "image_rgb" (its own seeded image, same size)."""
    out = []
    for i, (img, boxes, cls, masks) in enumerate(det_inputs()):
        rgb = np.floor(seeded(img.shape, 330 + i, "uniform") * 255.0)
        out.append((img, rgb, boxes, cls, masks))
    return out


@torch.no_grad()
def ema_teacher_state(model, fill_module, seed):
    """name -> value for every parameter and buffer of ``model`` as the EMA state iterates them: a
    mix of the model's own (name-hashed) fill and the fill at ``seed + EMA_MIX[2]`` for every
    entry the fill touches (identical on the reference and the product, whatever their module
    registration order), the model's own value elsewhere.  The second fill is made in place and
    the model's values are put back (no deepcopy: the product model holds module references)."""
    a, b, ds = EMA_MIX
    items = list(model.named_parameters()) + list(model.named_buffers())
    mine = {n: v.detach().clone() for n, v in items}
    fill_module(model, seed=seed + ds, dedup=True)
    theirs = {n: v.detach().clone() for n, v in items}
    for n, v in items:
        v.data.copy_(mine[n])
    out = {}
    for n, v in mine.items():
        w = theirs[n]
        out[n] = v if (not v.is_floating_point() or torch.equal(v, w)) else a * v + b * w
    return out


BASE_WEIGHTS = {"loss_class": 1, "loss_bbox": 5.0, "loss_giou": 2.0, "loss_class_dn": 0, "loss_bbox_dn": 0.0,
                "loss_giou_dn": 0.0, "loss_mask": 1.0, "loss_dice": 5.0, "loss_mask_dn": 0, "loss_dice_dn": 0}


def det_weight_dict(dec_layers):
    """configs/models/dino_r50.py:98-147: base weights, + "_enc", + "_{i}" for the aux layers."""
    w = dict(BASE_WEIGHTS)
    w.update({k + "_enc": v for k, v in BASE_WEIGHTS.items()})
    for i in range(dec_layers - 1):
        w.update({k + f"_{i}": v for k, v in BASE_WEIGHTS.items()})
    return w


def canonical_params(model):
    """(name, parameter) per distinct trainable parameter, named by its alphabetically first name
    (the detector's heads are registered twice: under the model and under its decoder)."""
    first = {}
    for n, p in model.named_parameters(remove_duplicate=False):
        if p.requires_grad and (id(p) not in first or n < first[id(p)][0]):
            first[id(p)] = (n, p)
    return sorted(first.values(), key=lambda x: x[0])


def seg_probes(model):
    """Forward hooks on the segmentation-feature branch (the concatenated level features, the
    mapping convs' output and the post LayerNorm's): (L2 norm, seeded projection) of each, for
    localising a difference between the reference and the product."""
    store = {}

    def stat(t):
        t = t.detach().double().cpu()
        g = torch.Generator().manual_seed(7)
        r = torch.randn(t.shape, generator=g, dtype=torch.float64)
        return [float(t.norm()), float((t * r).sum()), float(t.abs().sum())]

    hs = [model.mapping_fpn_features_for_seg.register_forward_pre_hook(
              lambda m, a: store.__setitem__("seg_in", stat(a[0]))),
          model.mapping_fpn_features_for_seg.register_forward_hook(
              lambda m, a, o: store.__setitem__("seg_mapped", stat(o))),
          model.mapping_fpn_features_for_seg[1].register_forward_hook(
              lambda m, a, o: store.__setitem__("seg_bn", stat(o))),
          model.post_layernorm.register_forward_hook(lambda m, a, o: store.__setitem__("seg_ln", stat(o)))]
    return store, hs
