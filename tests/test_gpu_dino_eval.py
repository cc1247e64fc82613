"""The vCLR detector's evaluation path on the GPU: the HIP NMS (irads_nms through ops.batched_nms)
against the CPU restatement of torchvision's nms / batched_nms (oracle/irads_ref.py), the inference
post-processing (DINO.postprocess: dino.py:923-947, 1204-1256, 41-105) against a CPU restatement
of those lines on the same raw outputs, and the end-to-end eval driver (data.TestMapper ->
model.eval() -> COCOEvaluatorCustom) on a synthetic COCO json.  torchvision and pycocotools are
absent: the NMS is pinned to the restated algorithm, the evaluator by tests/test_cpu_coco_eval.py."""
import json
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

from oracle import irads_ref as R  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _boxes(n, seed, labels=1):
    g = np.random.default_rng(seed)
    centers = g.uniform(0, 400, (max(1, n // 8), 2))  # clusters so that suppression happens
    c = centers[g.integers(0, len(centers), n)] + g.normal(0, 6, (n, 2))
    wh = g.uniform(8, 60, (n, 2))
    b = np.concatenate([c - wh / 2, c + wh / 2], 1).astype(np.float32)
    s = g.random(n).astype(np.float32)
    return b, s, g.integers(0, labels, n)


@pytest.mark.parametrize("n,labels,thr", [(300, 1, 0.7), (300, 3, 0.5), (4096, 5, 0.7), (1, 1, 0.7), (0, 1, 0.7)])
def test_batched_nms_vs_oracle(n, labels, thr):
    from irads import ops
    for seed in range(3):
        b, s, lab = _boxes(n, seed, labels)
        want = R.batched_nms_ref(b, s, lab, thr)
        got = ops.batched_nms(torch.as_tensor(b, device=DEV), torch.as_tensor(s, device=DEV),
                              torch.as_tensor(lab, device=DEV), thr).cpu().numpy()
        assert got.tolist() == want.tolist()


def test_nms_threshold_ties():
    """Pairs whose IoU is exactly the threshold are kept (suppression needs IoU > threshold)."""
    from irads import ops
    b = torch.tensor([[0, 0, 10, 10], [0, 0, 10, 5], [0, 0, 10, 2]], dtype=torch.float32, device=DEV)
    s = torch.tensor([0.9, 0.8, 0.7], device=DEV)
    # box 1: IoU with box 0 = 50 / 100 = 0.5, not > 0.5: kept; box 2: IoU .2 with box 0, .4 with box 1: kept
    assert ops.batched_nms(b, s, torch.zeros(3, dtype=torch.int64, device=DEV), 0.5).cpu().tolist() == [0, 1, 2]
    assert ops.batched_nms(b, s, torch.zeros(3, dtype=torch.int64, device=DEV), 0.45).cpu().tolist() == [0, 2]


def _postprocess_ref(output, sizes, out_hw, topk=300, thr=0.7):
    """dino.py:928-945 (scores, masks), 1204-1256 (nms_inference), 41-105 (detector_postprocess) on the
    CPU in fp32 as the reference computes, NMS by the oracle."""
    cls = output["pred_logits"].float().cpu()
    box = output["pred_boxes"].float().cpu()
    msk = output["pred_masks"].float().cpu()
    ms = ((msk > 0) * msk.sigmoid()).sum((2, 3)) / ((msk > 0).sum((2, 3)) + 1e-10)
    x = torch.sqrt(cls.sigmoid() * ms.unsqueeze(-1)).clamp(0, 1)
    avg = torch.log(x.clamp(min=1e-3) / (1 - x).clamp(min=1e-3))
    bs, nq, nc = avg.shape
    prob = avg.sigmoid().view(bs, -1)
    out = []
    for i in range(bs):
        pre = prob[i].topk(min(topk, nq * nc)).indices
        q, lab = pre // nc, pre % nc
        cx, cy, w, h = box[i][q].unbind(-1)
        b = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], -1)
        keep = torch.as_tensor(R.batched_nms_ref(b.numpy(), prob[i][pre].numpy(), lab.numpy(), thr))
        hi, wi = sizes[i]
        H, W = out_hw[i]
        b = b[keep] * torch.tensor([wi, hi, wi, hi], dtype=torch.float32) * torch.tensor(
            [W / wi, H / hi, W / wi, H / hi], dtype=torch.float32)
        b = torch.stack([b[:, 0].clamp(0, W), b[:, 1].clamp(0, H), b[:, 2].clamp(0, W), b[:, 3].clamp(0, H)], 1)
        ok = (b[:, 2] > b[:, 0]) & (b[:, 3] > b[:, 1])
        out.append((b[ok], prob[i][pre][keep][ok]))
    return out


def test_postprocess_vs_reference_lines():
    from projects.vCLR_deformable_mask.configs.dino_r50 import build_model
    model = build_model(num_classes=2, num_queries=40, enc_layers=1, dec_layers=1, dn_number=4,
                        consistency=False).to(DEV).eval()
    g = torch.Generator().manual_seed(0)
    bs, nq, nc, h, w = 2, 40, 2, 24, 30
    c = torch.rand(bs, nq, 2, generator=g) * 0.8 + 0.1
    wh = torch.rand(bs, nq, 2, generator=g) * 0.3 + 0.05
    output = {"pred_logits": torch.randn(bs, nq, nc, generator=g).to(DEV),
              "pred_boxes": torch.cat([c, wh], -1).to(DEV),
              "pred_masks": torch.randn(bs, nq, h, w, generator=g).to(DEV)}
    sizes = [(190, 240), (170, 236)]
    batched = [{"height": 380, "width": 480}, {"height": 300, "width": 420}]
    got = model.postprocess(output, batched, sizes, topk=60)
    want = _postprocess_ref(output, sizes, [(380, 480), (300, 420)], topk=60)
    for r, (wb, ws) in zip(got, want):
        inst = r["instances"]
        assert inst["pred_boxes"].shape[0] == wb.shape[0] > 0
        torch.testing.assert_close(inst["pred_boxes"].cpu(), wb, rtol=1e-5, atol=1e-3)
        torch.testing.assert_close(inst["scores"].cpu(), ws, rtol=1e-5, atol=1e-6)
        assert inst["pred_masks"].dtype == torch.bool and inst["pred_masks"].shape[1:] == tuple(inst["image_size"])
    # the masks: bilinear to the output size, > 0
    i0 = got[0]["instances"]
    assert i0["pred_masks"].shape[0] == i0["scores"].shape[0]


def test_eval_driver_end_to_end(tmp_path):
    """A reduced DINO (1 + 1 layers, 30 queries) in eval mode over a two-image synthetic COCO json:
    every stat of COCOEvaluatorCustom's 23 for boxes and masks is a percentage or nan."""
    from PIL import Image
    from detrex.evaluation.coco import METRICS_VCLR
    from projects.vCLR_deformable_mask.configs.dino_r50 import build_model
    from projects.vCLR_deformable_mask.data import TestMapper, filter_empty, load_coco_json
    from projects.vCLR_deformable_mask.evaluate import evaluate
    g = np.random.default_rng(0)
    ims, anns = [], []
    for i, (hh, ww) in enumerate([(96, 128), (120, 100)]):
        Image.fromarray(g.integers(0, 255, (hh, ww, 3), dtype=np.uint8)).save(tmp_path / f"{i}.png")
        ims.append({"id": i + 1, "file_name": f"{i}.png", "height": hh, "width": ww})
        for k in range(3):
            x, y = float(g.integers(0, ww - 30)), float(g.integers(0, hh - 30))
            anns.append({"id": len(anns) + 1, "image_id": i + 1, "category_id": 1, "bbox": [x, y, 25.0, 20.0],
                         "area": 500.0, "iscrowd": 0,
                         "segmentation": [[x, y, x + 25, y, x + 25, y + 20, x, y + 20]]})
    (tmp_path / "ann.json").write_text(json.dumps({"images": ims, "annotations": anns,
                                                   "categories": [{"id": 1, "name": "object"}]}))
    dicts, meta = load_coco_json(str(tmp_path / "ann.json"), str(tmp_path))
    dicts = filter_empty(dicts)
    torch.manual_seed(0)
    model = build_model(num_classes=1, num_queries=30, enc_layers=1, dec_layers=1, dn_number=4,
                        consistency=False).to(DEV)
    res = evaluate(model, dicts, meta, mapper=TestMapper(min_size=160, max_size=320))
    assert set(res) == {"bbox", "segm"}
    for task in res.values():
        for m in METRICS_VCLR:
            v = task[m]
            assert np.isnan(v) or 0.0 <= v <= 100.0
    assert model.training  # evaluate() restores the mode it found


def test_train_mapper_feeds_the_training_step(tmp_path):
    """COCO json -> data.TrainMapper (OursDatasetMapper's augmentations, instances with bool masks) ->
    train_net.run_step (EMA teacher, strong view, DINO + consistency criteria, clip, AdamW, EMA update)
    on a reduced model: finite losses, the weights and the EMA state move."""
    from PIL import Image
    from projects.vCLR_deformable_mask import train_net
    from projects.vCLR_deformable_mask.configs.dino_r50 import build_model
    from projects.vCLR_deformable_mask.data import TrainMapper, filter_empty, load_coco_json
    g = np.random.default_rng(1)
    ims, anns = [], []
    for i, (hh, ww) in enumerate([(120, 160), (100, 150)]):
        Image.fromarray(g.integers(0, 255, (hh, ww, 3), dtype=np.uint8)).save(tmp_path / f"{i}.png")
        ims.append({"id": i + 1, "file_name": f"{i}.png", "height": hh, "width": ww})
        for k in range(4):
            x, y = float(g.integers(0, ww - 40)), float(g.integers(0, hh - 40))
            anns.append({"id": len(anns) + 1, "image_id": i + 1, "category_id": 7, "bbox": [x, y, 35.0, 30.0],
                         "area": 1050.0, "iscrowd": 0,
                         "segmentation": [[x, y, x + 35, y, x + 35, y + 30, x, y + 30]]})
    (tmp_path / "ann.json").write_text(json.dumps({"images": ims, "annotations": anns,
                                                   "categories": [{"id": 7, "name": "object"}]}))
    dicts, meta = load_coco_json(str(tmp_path / "ann.json"), str(tmp_path))
    dicts = filter_empty(dicts)
    np.random.seed(0)
    import random
    random.seed(0)
    batched = [TrainMapper()(d) for d in dicts]
    for b in batched:
        inst = b["instances"]
        assert inst["gt_masks"].dtype == torch.bool and inst["gt_boxes"].shape[0] >= 1
        assert tuple(b["image"].shape[1:]) == tuple(inst["image_size"]) == tuple(b["image_rgb"].shape[1:])
    torch.manual_seed(0)
    model = build_model(num_classes=1, num_queries=30, enc_layers=1, dec_layers=1, dn_number=4).to(DEV).train()
    updater = train_net.build_ema(model, decay=0.999)
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4, weight_decay=1e-4)
    w0 = model.class_embed[0].weight.detach().clone()
    ema0 = {k: v.detach().clone() for k, v in updater.state.state.items()} if hasattr(updater.state, "state") else None
    for _ in range(2):
        total, losses = train_net.run_step(model, opt, batched, {"max_norm": 0.1, "norm_type": 2}, updater)
        assert torch.isfinite(total) and all(torch.isfinite(v) for v in losses.values())
    assert "loss_sim" in losses  # the consistency criterion ran against the EMA teacher
    assert not torch.equal(model.class_embed[0].weight, w0)
    if ema0 is not None:
        assert any(not torch.equal(updater.state.state[k], ema0[k]) for k in ema0)
