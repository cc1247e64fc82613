"""Localise a product / reference difference in the vCLR DINO detector step (debugging aid).

    python scripts/dino_det_dump.py product   out.npz   # on a GPU box: the product, fp64
    python scripts/dino_det_dump.py reference out.npz   # here: the reference on the CPU, fp64
    python scripts/dino_det_dump.py compare a.npz b.npz

Both sides run tests/test_gpu_dino_detector.py's case (same weights, inputs and replayed draws)
and keep the outputs of the backbone, neck, transformer and segmentation branch, the mask
predictions and the loss dict."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ir-ads_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def hooks(model, store):
    def keep(name):
        def f(m, a, o):
            if isinstance(o, dict):
                for k, v in o.items():
                    store[f"{name}.{k}"] = v.detach().double().cpu().numpy()
            elif isinstance(o, (list, tuple)):
                for i, v in enumerate(o):
                    if torch.is_tensor(v):
                        store[f"{name}.{i}"] = v.detach().double().cpu().numpy()
            else:
                store[name] = o.detach().double().cpu().numpy()
        return f
    hs = [model.backbone.register_forward_hook(keep("backbone")),
          model.neck.register_forward_hook(keep("neck")),
          model.transformer.register_forward_hook(keep("transformer")),
          model.mapping_fpn_features_for_seg.register_forward_pre_hook(
              lambda m, a: store.__setitem__("seg_in", a[0].detach().double().cpu().numpy())),
          model.mapping_fpn_features_for_seg.register_forward_hook(keep("seg_mapped")),
          model.post_layernorm.register_forward_hook(keep("seg_ln"))]
    cnt = [0]

    def pos_hook(m, a, o):
        store[f"pos{cnt[0]}"] = o.detach().double().cpu().numpy()
        store[f"posmask{cnt[0]}"] = a[0].detach().double().cpu().numpy()
        cnt[0] += 1
    hs.append(model.position_embedding.register_forward_hook(pos_hook))
    for i, m in enumerate(model.mask_embed):
        hs.append(m.register_forward_hook(keep(f"mask_embed{i}")))
    for i, layer in enumerate(model.transformer.encoder.layers):
        at = layer.attentions[0]
        hs.append(layer.register_forward_hook(keep(f"enc{i}.out")))
        hs.append(at.register_forward_hook(keep(f"enc{i}.msda_module_out")))
        for name in ("sampling_offsets", "attention_weights", "value_proj"):
            hs.append(getattr(at, name).register_forward_hook(keep(f"enc{i}.{name}")))
        hs.append(at.output_proj.register_forward_pre_hook(
            lambda m, a, i=i: store.__setitem__(f"enc{i}.msda_core", a[0].detach().double().cpu().numpy())))
    return hs


def product(out):
    from golden_util import Fixture
    from dino_det_case import DET_CFG, DET_FILL_SEED, DET_NUM_POINTS, ReplayRNG, det_inputs
    from fill import fill_module
    from projects.vCLR_deformable_mask.configs.dino_r50 import build_model
    dev = torch.device("cuda", 0)
    dtype = torch.float64
    fx = Fixture("dino_detector_step.npz")
    model = build_model(**DET_CFG, device="cuda")
    model.criterion.num_points = DET_NUM_POINTS
    fill_module(model, seed=DET_FILL_SEED, dedup=True)
    model = model.to(dev).to(dtype).train()
    rng = ReplayRNG([fx[f"draw_{i}"] for i in range(int(fx["n_draws"]))])
    model.rng = model.criterion.rng = rng
    batched = []
    for img, boxes, cls, masks in det_inputs():
        inst = {"image_size": tuple(img.shape[1:]), "gt_boxes": torch.as_tensor(boxes, dtype=dtype, device=dev),
                "gt_classes": torch.as_tensor(cls, device=dev), "gt_masks": torch.as_tensor(masks, device=dev)}
        batched.append({"image": torch.as_tensor(img, dtype=dtype), "instances": inst})
    store = {}
    hs = hooks(model, store)
    images, _ = model.preprocess_image(batched)
    B, _, H, W = images.shape
    img_masks = images.new_ones(B, H, W)
    for i, x in enumerate(batched):
        ih, iw = x["instances"]["image_size"]
        img_masks[i, :ih, :iw] = 0
    losses = model.forward_student(batched, images, img_masks)
    for h in hs:
        h.remove()
    for k, v in losses.items():
        store["loss." + k] = np.array(float(v.detach()))
    np.savez(out, **store)
    print("saved", len(store), "arrays")


def reference(out):
    import gen_golden as G
    from dino_det_case import ReplayRNG
    from golden_util import Fixture
    fx = Fixture("dino_detector_step.npz")
    L = __import__("ref_import").load_dino_detector()
    store = {}
    orig = G._det_reference_model

    def model_with_hooks(L_, dtype):
        m = orig(L_, dtype)
        hooks(m, store)
        return m
    G._det_reference_model = model_with_hooks
    losses, _, _ = G._det_reference_step(L, torch.float64, ReplayRNG([fx[f"draw_{i}"] for i in range(int(fx["n_draws"]))]))
    losses.pop("_probes", None)
    for k, v in losses.items():
        store["loss." + k] = np.array(float(v.detach()))
    np.savez(out, **store)
    print("saved", len(store), "arrays")


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    for k in A.files:
        if k not in Bz.files:
            print(f"{k:40s} only in {a}")
            continue
        x, y = A[k], Bz[k]
        if x.shape != y.shape:
            print(f"{k:40s} shape {x.shape} vs {y.shape}")
            continue
        d = np.abs(x - y)
        fin = np.isfinite(y)
        rel = float(np.sqrt((d[fin] ** 2).sum()) / max(np.sqrt((y[fin] ** 2).sum()), 1e-300))
        idx = np.unravel_index(np.argmax(np.where(fin, d, 0)), d.shape) if d.size else ()
        print(f"{k:40s} rel_l2 {rel:.3e}  max_abs {float(np.where(fin, d, 0).max()) if d.size else 0:.3e} at {idx}")


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "product":
        product(sys.argv[2])
    elif mode == "reference":
        reference(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
