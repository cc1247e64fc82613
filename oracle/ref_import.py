"""Container-only loader for the IR-ADS *reference* Python modules.

TEST INFRASTRUCTURE ONLY.  Used solely by ``oracle/gen_golden.py`` to produce the
golden fixtures under ``tests/golden/``.  ``/root/reference`` never ships to the GPU
box; nothing in the product, in ``bench.py`` or in the ``-m gpu`` tests imports this.

The reference modules are loaded by file path.  Their missing
third-party symbols (mmcv 2.0.0rc4, mmengine 0.10.7, mmseg 1.2.2, timm 0.4.12,
fvcore, geotorch) are registered as small stand-ins whose semantics follow those
packages as the reference uses them:

* ``build_norm_layer(dict(type='LN'), C)`` -> ``('ln', nn.LayerNorm(C))`` (eps 1e-5)
* ``build_conv_layer(cfg, ...)`` -> ``nn.Conv2d(...)``
* mmcv ``FFN``: ``layers = Seq(Seq(Linear, GELU, Dropout), Linear, Dropout)``,
  ``forward(x, identity) = identity + dropout_layer(layers(x))``
* ``build_dropout(DropPath)`` -> timm DropPath
* geotorch.orthogonal -> no-op (only the non-diagonal LightSB path uses it: parity unpinned)
* ``modeling.sb_modules.MyMixtureSameFamily.MixtureSameFamily`` ->
  ``torch.distributions.MixtureSameFamily``

The mmcv/mmengine/timm arithmetic is therefore "parity unpinned" (no reference test
covers it); PyTorch's own LayerNorm / Linear / GELU / grid_sample are the arithmetic.
"""
import importlib.util
import sys
import types

import torch
import torch.nn as nn

REF = "/root/reference"


def _mod(name, **attrs):
    m = sys.modules.get(name) or types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _DropPath(nn.Module):
    def __init__(self, drop_prob=0.0):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        if self.drop_prob == 0.0 or not self.training:
            return x
        kp = 1 - self.drop_prob
        shape = (x.shape[0],) + (1,) * (x.ndim - 1)
        r = kp + torch.rand(shape, dtype=x.dtype, device=x.device)
        r.floor_()
        return x.div(kp) * r


def _build_dropout(cfg):
    cfg = dict(cfg)
    t = cfg.pop("type")
    if t == "DropPath":
        return _DropPath(cfg.get("drop_prob", 0.0))
    if t == "Dropout":
        return nn.Dropout(cfg.get("drop_prob", 0.0))
    raise ValueError(t)


class _FFN(nn.Module):
    def __init__(self, embed_dims=256, feedforward_channels=1024, num_fcs=2,
                 act_cfg=dict(type="ReLU", inplace=True), ffn_drop=0.0,
                 dropout_layer=None, add_identity=True, init_cfg=None, **kw):
        super().__init__()
        assert num_fcs == 2
        act = {"GELU": nn.GELU(), "ReLU": nn.ReLU(True)}[act_cfg["type"]]
        self.layers = nn.Sequential(
            nn.Sequential(nn.Linear(embed_dims, feedforward_channels), act, nn.Dropout(ffn_drop)),
            nn.Linear(feedforward_channels, embed_dims),
            nn.Dropout(ffn_drop),
        )
        self.dropout_layer = _build_dropout(dropout_layer) if dropout_layer else nn.Identity()
        self.add_identity = add_identity

    def forward(self, x, identity=None):
        out = self.layers(x)
        if not self.add_identity:
            return self.dropout_layer(out)
        if identity is None:
            identity = x
        return identity + self.dropout_layer(out)


class _BaseModule(nn.Module):
    def __init__(self, init_cfg=None):
        super().__init__()
        self.init_cfg = init_cfg


def _build_norm_layer(cfg, num_features):
    assert cfg["type"] == "LN", cfg
    return "ln", nn.LayerNorm(num_features)


def _to_2tuple(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, x)


class _Registry:
    def register_module(self, *a, **k):
        return lambda cls: cls


def _install_standins():
    _mod("mmcv")
    _mod("mmcv.cnn", build_norm_layer=_build_norm_layer,
         build_conv_layer=lambda cfg, *a, **k: nn.Conv2d(*a, **k))
    _mod("mmcv.cnn.bricks")
    _mod("mmcv.cnn.bricks.transformer", FFN=_FFN, build_dropout=_build_dropout)
    _mod("mmengine")
    _mod("mmengine.logging", print_log=lambda *a, **k: None)
    _mod("mmengine.model", BaseModule=_BaseModule, ModuleList=nn.ModuleList)
    _mod("mmengine.model.weight_init", trunc_normal_=nn.init.trunc_normal_,
         constant_init=lambda m, val, bias=0: None, trunc_normal_init=lambda m, std, bias=0: None)
    _mod("mmengine.runner", CheckpointLoader=None)
    _mod("mmengine.utils", to_2tuple=_to_2tuple)
    _mod("mmseg")
    _mod("mmseg.registry", MODELS=_Registry())
    _mod("timm")
    _mod("timm.models")
    _mod("timm.models.layers", DropPath=_DropPath)
    _mod("fvcore")
    _mod("fvcore.nn", flop_count_table=None, FlopCountAnalysis=None)
    _mod("geotorch", orthogonal=lambda *a, **k: None)
    _mod("modeling")
    _mod("modeling.sb_modules")
    _mod("modeling.sb_modules.MyMixtureSameFamily",
         MixtureSameFamily=torch.distributions.MixtureSameFamily)
    # placeholder so MultiScaleDeformableAttention is not replaced by the dummy class;
    # on CPU tensors the module takes its PyTorch path (multi_scale_deform_attn.py:341-353)
    for p in ("detrex", "detrex.layers"):
        _mod(p)
    _mod("detrex._C")
    for p in ("semseg", "semseg.models", "semseg.models.backbones", "semseg.models.heads",
              "semseg.models.layers", "modules"):
        m = _mod(p)
        m.__path__ = []


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, f"{REF}/{rel}")
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m


_LOADED = {}


def load_reference():
    """Return a namespace with the reference's hot-path modules."""
    if _LOADED:
        return types.SimpleNamespace(**_LOADED)
    _install_standins()
    common = _load("semseg.models.layers.common", "semseg/models/layers/common.py")
    init = _load("semseg.models.layers.initialize", "semseg/models/layers/initialize.py")
    layers = sys.modules["semseg.models.layers"]
    for m in (common, init):
        for k in dir(m):
            if not k.startswith("_"):
                setattr(layers, k, getattr(m, k))
    embed = _load("semseg.models.backbones.embed", "semseg/models/backbones/embed.py")
    swin = _load("semseg.models.backbones.swin", "semseg/models/backbones/swin.py")
    bb = sys.modules["semseg.models.backbones"]
    bb.SwinTransformer = swin.SwinTransformer
    seg = _load("semseg.models.heads.segformer", "semseg/models/heads/segformer.py")
    heads = sys.modules["semseg.models.heads"]
    heads.SegFormerHead = seg.SegFormerHead
    heads.LightHamHead = None
    heads.UPerHead = None
    base = _load("semseg.models.base", "semseg/models/base.py")
    cmnext = _load("semseg.models.cmnext", "semseg/models/cmnext.py")
    msda = _load("detrex.layers.multi_scale_deform_attn", "detrex/layers/multi_scale_deform_attn.py")
    sb = _load("modules.sb", "modules/sb.py")
    metrics = _load("semseg.metrics", "semseg/metrics.py")
    _LOADED.update(swin=swin, embed=embed, segformer=seg, base=base, cmnext=cmnext,
                   msda=msda, sb=sb, metrics=metrics)
    return types.SimpleNamespace(**_LOADED)


def load_dino():
    """The vCLR DINO transformer (projects/vCLR_deformable_mask/modeling/dino_transformer.py) on
    the reference's own detrex layers.  Stand-ins: fairscale's ``checkpoint_wrapper`` (identity;
    the reference discards its result anyway, :74-77) and an empty ``torchvision`` (only
    detrex/utils/misc.py's unused box helpers need it).  MSDA takes its CPU PyTorch path."""
    ref = load_reference()
    if "dino" in _LOADED:
        return ref
    _mod("fairscale")
    _mod("fairscale.nn")
    _mod("fairscale.nn.checkpoint", checkpoint_wrapper=lambda m, *a, **k: m)
    if importlib.util.find_spec("torchvision") is None:
        _mod("torchvision")
    lay = sys.modules["detrex.layers"]
    for name, rel in (("transformer", "transformer.py"), ("attention", "attention.py"), ("mlp", "mlp.py"),
                      ("position_embedding", "position_embedding.py")):
        m = _load(f"detrex.layers.{name}", f"detrex/layers/{rel}")
        for k in dir(m):
            if not k.startswith("_"):
                setattr(lay, k, getattr(m, k))
    lay.MultiScaleDeformableAttention = _LOADED["msda"].MultiScaleDeformableAttention
    misc = _load("detrex.utils.misc", "detrex/utils/misc.py")
    _mod("detrex.utils", inverse_sigmoid=misc.inverse_sigmoid)
    dino = _load("vclr_dino_transformer", "projects/vCLR_deformable_mask/modeling/dino_transformer.py")
    _LOADED.update(dino=dino, detrex_layers=lay)
    return types.SimpleNamespace(**_LOADED)


def load_val_mm():
    """The reference's evaluation driver val_mm.py (evaluate / evaluate_msf, val_mm.py:64-120).
    Its module-level imports that the evaluation functions never use (datasets, augmentations,
    the utils' DDP / logging helpers) are empty stand-ins; semseg.metrics is the reference's."""
    ref = load_reference()
    if "val_mm" in _LOADED:
        return ref
    _mod("semseg.datasets").__path__ = []
    _mod("semseg.augmentations_mm", get_val_augmentation=None)
    _mod("semseg.utils").__path__ = []
    _mod("semseg.utils.utils", fix_seeds=None, setup_cudnn=None, cleanup_ddp=None, setup_ddp=None,
         get_logger=None, cal_flops=None, print_iou=None)
    _LOADED.update(val_mm=_load("reference_val_mm", "val_mm.py"))
    return types.SimpleNamespace(**_LOADED)


if __name__ == "__main__":
    r = load_reference()
    print(sorted(vars(r)))


# ---------------------------------------------------------------------------------------------
# vCLR DINO detector (projects/vCLR_deformable_mask/modeling/dino.py + its criteria) for the
# reduced training-step fixture.  Stand-ins, restating the published detectron2 0.6 / fvcore /
# torchvision pieces the detector path uses (their arithmetic is therefore parity unpinned):
#   detectron2.layers: Conv2d(norm=, activation=), FrozenBatchNorm2d (eps 1e-5), get_norm,
#     CNNBlockBase, ShapeSpec; detectron2.modeling.backbone.Backbone;
#   detectron2.structures: Boxes (.tensor), ImageList.from_tensors (bottom/right zero padding),
#     Instances (image_size + fields);
#   detectron2.projects.point_rend.point_features: point_sample (grid_sample of 2p - 1) and
#     get_uncertain_point_coords_with_randomness (uniform oversampling, top-k uncertainty,
#     uniform fill);
#   fvcore.nn.weight_init.c2_msra_fill (the fixture overwrites every weight anyway);
#   torchvision._is_tracing -> False, torchvision.ops.boxes.box_area ((x1 - x0)(y1 - y0));
#   detrex.utils dist helpers for one process;
#   detrex.modeling.ema, NMS, event storage, image-format conversion: unused by the training
#   forward (None).
# The reference calls .cuda() / .to("cuda") inside prepare_for_cdn and the dn criterion; for
# this CPU-only generation those become no-ops (patched only while the fixture is made).
class _D2Conv2d(nn.Conv2d):
    def __init__(self, *args, **kwargs):
        norm = kwargs.pop("norm", None)
        activation = kwargs.pop("activation", None)
        super().__init__(*args, **kwargs)
        self.norm, self.activation = norm, activation

    def forward(self, x):
        x = torch.nn.functional.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation,
                                       self.groups)
        if self.norm is not None:
            x = self.norm(x)
        if self.activation is not None:
            x = self.activation(x)
        return x


class _FrozenBN(nn.Module):
    def __init__(self, num_features, eps=1e-5):
        super().__init__()
        self.num_features, self.eps = num_features, eps
        self.register_buffer("weight", torch.ones(num_features))
        self.register_buffer("bias", torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features) - eps)

    def forward(self, x):
        scale = self.weight * (self.running_var + self.eps).rsqrt()
        bias = self.bias - self.running_mean * scale
        return x * scale.reshape(1, -1, 1, 1).to(x.dtype) + bias.reshape(1, -1, 1, 1).to(x.dtype)


class _CNNBlockBase(nn.Module):
    def __init__(self, in_channels, out_channels, stride):
        super().__init__()
        self.in_channels, self.out_channels, self.stride = in_channels, out_channels, stride

    def freeze(self):
        for p in self.parameters():
            p.requires_grad = False
        return self


def _get_norm(norm, out_channels):
    if norm is None or norm == "":
        return None
    return {"FrozenBN": _FrozenBN, "BN": nn.BatchNorm2d}[norm](out_channels)


class _Backbone(nn.Module):
    @property
    def size_divisibility(self):
        return 0


class _Boxes:
    def __init__(self, tensor):
        self.tensor = tensor


class _ImageList:
    def __init__(self, tensor, image_sizes):
        self.tensor, self.image_sizes = tensor, image_sizes

    @staticmethod
    def from_tensors(tensors, size_divisibility=0, pad_value=0.0):
        H = max(t.shape[-2] for t in tensors)
        W = max(t.shape[-1] for t in tensors)
        out = tensors[0].new_full((len(tensors), tensors[0].shape[0], H, W), pad_value)
        for o, t in zip(out, tensors):
            o[:, :t.shape[-2], :t.shape[-1]].copy_(t)
        return _ImageList(out, [tuple(t.shape[-2:]) for t in tensors])


class _Instances:
    def __init__(self, image_size, **fields):
        self.image_size = image_size
        for k, v in fields.items():
            setattr(self, k, v)

    def to(self, device):
        return self


def _point_sample(input, point_coords, **kwargs):
    add_dim = point_coords.dim() == 3
    if add_dim:
        point_coords = point_coords.unsqueeze(2)
    out = torch.nn.functional.grid_sample(input, 2.0 * point_coords - 1.0, **kwargs)
    return out.squeeze(3) if add_dim else out


def _uncertain_points(coarse_logits, uncertainty_func, num_points, oversample_ratio, importance_sample_ratio):
    num_boxes = coarse_logits.shape[0]
    num_sampled = int(num_points * oversample_ratio)
    point_coords = torch.rand(num_boxes, num_sampled, 2, device=coarse_logits.device)
    point_logits = _point_sample(coarse_logits, point_coords, align_corners=False)
    point_uncertainties = uncertainty_func(point_logits)
    num_uncertain = int(importance_sample_ratio * num_points)
    num_random = num_points - num_uncertain
    idx = torch.topk(point_uncertainties[:, 0, :], k=num_uncertain, dim=1)[1]
    shift = num_sampled * torch.arange(num_boxes, dtype=torch.long, device=coarse_logits.device)
    idx += shift[:, None]
    point_coords = point_coords.view(-1, 2)[idx.view(-1), :].view(num_boxes, num_uncertain, 2)
    if num_random > 0:
        point_coords = torch.cat([point_coords, torch.rand(num_boxes, num_random, 2, device=coarse_logits.device)], 1)
    return point_coords


def _c2_msra_fill(m):
    nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
    if m.bias is not None:
        nn.init.constant_(m.bias, 0)


def _pkg(name):
    m = _mod(name)
    m.__path__ = []
    return m


def load_dino_detector():
    """The reference DINO detector, its criteria, matcher, ResNet and ChannelMapper (see above)."""
    import collections
    ref = load_dino()
    if "dino_det" in _LOADED:
        return ref
    _ShapeSpec = collections.namedtuple("ShapeSpec", ["channels", "height", "width", "stride"],
                                        defaults=(None, None, None, None))
    for p in ("detectron2", "detectron2.utils", "detectron2.data", "detectron2.modeling", "detectron2.projects",
              "detectron2.projects.point_rend"):
        _pkg(p)
    _mod("detectron2.layers", Conv2d=_D2Conv2d, FrozenBatchNorm2d=_FrozenBN, get_norm=_get_norm,
         CNNBlockBase=_CNNBlockBase, ShapeSpec=_ShapeSpec, DeformConv=None, ModulatedDeformConv=None,
         cat=torch.cat).__path__ = []
    _mod("detectron2.layers.nms", batched_nms=None)
    _mod("detectron2.modeling.backbone", Backbone=_Backbone)
    _mod("detectron2.structures", Boxes=_Boxes, ImageList=_ImageList, Instances=_Instances, ROIMasks=None)
    _mod("detectron2.utils.events", get_event_storage=None)
    _mod("detectron2.data.detection_utils", convert_image_to_rgb=None)
    _mod("detectron2.projects.point_rend.point_features", point_sample=_point_sample,
         get_uncertain_point_coords_with_randomness=_uncertain_points)
    _pkg("fvcore")
    _mod("fvcore.nn.weight_init", c2_msra_fill=_c2_msra_fill)
    sys.modules["fvcore.nn"].weight_init = sys.modules["fvcore.nn.weight_init"]
    tv = _mod("torchvision")
    tv._is_tracing = lambda: False
    tv.__path__ = []
    _pkg("torchvision.ops")
    _mod("torchvision.ops.boxes", box_area=lambda b: (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]))
    import torch.distributed as tdist
    du = sys.modules["detrex.utils"]
    du.get_world_size = lambda: tdist.get_world_size() if tdist.is_available() and tdist.is_initialized() else 1
    du.is_dist_avail_and_initialized = lambda: tdist.is_available() and tdist.is_initialized()
    lay = sys.modules["detrex.layers"]
    for name, rel in (("box_ops", "box_ops.py"), ("conv", "conv.py"), ("shape_spec", "shape_spec.py")):
        m = _load(f"detrex.layers.{name}", f"detrex/layers/{rel}")
        for k in dir(m):
            if not k.startswith("_"):
                setattr(lay, k, getattr(m, k))
    _pkg("detrex.modeling")
    _mod("detrex.modeling.ema", apply_model_ema_and_restore=None)
    sys.modules["detrex.modeling"].ema = sys.modules["detrex.modeling.ema"]
    _pkg("detrex.modeling.criterion")
    crit = _load("detrex.modeling.criterion.criterion", "detrex/modeling/criterion/criterion.py")
    sys.modules["detrex.modeling.criterion"].SetCriterion = crit.SetCriterion
    matcher = _load("detrex.modeling.matcher.matcher", "detrex/modeling/matcher/matcher.py")
    neck = _load("detrex.modeling.neck.channel_mapper", "detrex/modeling/neck/channel_mapper.py")
    resnet = _load("detrex.modeling.backbone.resnet", "detrex/modeling/backbone/resnet.py")
    pkg = _pkg("vclr_modeling")
    pkg.__path__ = [f"{REF}/projects/vCLR_deformable_mask/modeling"]
    for name in ("misc", "two_stage_criterion", "dn_criterion", "dino"):
        spec = importlib.util.spec_from_file_location(f"vclr_modeling.{name}",
                                                      f"{REF}/projects/vCLR_deformable_mask/modeling/{name}.py")
        m = importlib.util.module_from_spec(spec)
        sys.modules[f"vclr_modeling.{name}"] = m
        spec.loader.exec_module(m)
        _LOADED[f"vclr_{name}"] = m
    _LOADED.update(dino_det=sys.modules["vclr_modeling.dino"], matcher=matcher, neck=neck, resnet=resnet,
                   criterion=sys.modules["vclr_modeling.dn_criterion"], ShapeSpec=_ShapeSpec,
                   ImageList=_ImageList, Instances=_Instances, Boxes=_Boxes)
    return types.SimpleNamespace(**_LOADED)


class _HookBase:
    """detectron2.engine.train_loop.HookBase (the EMA module subclasses it; never driven here)."""


def load_dino_train():
    """load_dino_detector() plus the pieces of the reference's full training forward (DINO.forward,
    dino.py:278-303): detrex/modeling/ema.py itself (EMAState, apply_model_ema_and_restore; its
    detectron2 HookBase import stood in) bound as the `ema` module dino.py calls, and
    ConsisCriterion.py."""
    ref = load_dino_detector()
    if "consis" in _LOADED:
        return types.SimpleNamespace(**_LOADED)
    _pkg("detectron2.engine")
    _mod("detectron2.engine.train_loop", HookBase=_HookBase)
    ema = _load("detrex.modeling.ema_reference", "detrex/modeling/ema.py")
    _LOADED["dino_det"].ema = ema
    spec = importlib.util.spec_from_file_location(
        "vclr_modeling.ConsisCriterion", f"{REF}/projects/vCLR_deformable_mask/modeling/ConsisCriterion.py")
    m = importlib.util.module_from_spec(spec)
    sys.modules["vclr_modeling.ConsisCriterion"] = m
    spec.loader.exec_module(m)
    _LOADED.update(ema=ema, consis=m)
    del ref
    return types.SimpleNamespace(**_LOADED)
