"""vCLR detector evaluation without detectron2: the reference's do_test (train_net.py, detectron2
inference_on_dataset with the config's test loader and evaluator,
configs/dino-resnet/deformable_train_voc_eval_nonvoc.py:76-99).  The COCO json's images go through
the test mapper (ResizeShortestEdge 800 / 1333, data.TestMapper), the model in eval mode returns the
post-processed detections (DINO.postprocess: mask-weighted scores, top 300, NMS on the HIP kernel,
boxes and masks at the original size), and COCOEvaluatorCustom reports the 23 AP / AR numbers for
boxes and masks at max_dets_per_image [1, 10, 20, 30, 50, 100, 300, 900].

    python -m projects.vCLR_deformable_mask.evaluate --json ann.json --images img_dir \\
        [--weights model.pth] [--num-queries 2000] [--limit N]        (cwd: ir-ads_amd)
"""
import argparse
import json
import time

import torch

from detrex.evaluation.coco import MAX_DETS_VCLR, COCOEvaluatorCustom

from .data import TestMapper, filter_empty, load_coco_json


def evaluate(model, dicts, meta, batch_size=1, max_dets=MAX_DETS_VCLR, mapper=None, log_every=0):
    """Run ``model`` (eval mode) over ``dicts`` and evaluate against ``meta["json"]``."""
    mapper = mapper or TestMapper()
    inv = {v: k for k, v in meta["thing_dataset_id_to_contiguous_id"].items()}
    ev = COCOEvaluatorCustom(meta["json"], max_dets, contiguous_to_dataset_id=inv)
    was_training = model.training
    model.eval()
    t0 = time.time()
    with torch.no_grad():
        for i in range(0, len(dicts), batch_size):
            batch = [mapper(d) for d in dicts[i:i + batch_size]]
            ev.process(batch, model(batch))
            if log_every and (i // batch_size) % log_every == 0:
                print(f"[eval] {i + len(batch)}/{len(dicts)} images, {time.time() - t0:.1f} s", flush=True)
    model.train(was_training)
    return ev.evaluate(img_ids=[d["image_id"] for d in dicts])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", required=True)
    ap.add_argument("--images", required=True)
    ap.add_argument("--weights", default=None, help="state dict (torch.save of model.state_dict())")
    ap.add_argument("--num-queries", type=int, default=2000)  # the config's model.num_queries
    ap.add_argument("--limit", type=int, default=0)
    ap.add_argument("--batch-size", type=int, default=1)
    args = ap.parse_args()
    from .configs.dino_r50 import build_model
    dicts, meta = load_coco_json(args.json, args.images)
    dicts = filter_empty(dicts)  # dataloader.test ... filter_empty=True
    if args.limit:
        dicts = dicts[:args.limit]
    model = build_model(num_classes=len(meta["thing_classes"]), num_queries=args.num_queries, consistency=False)
    if args.weights:
        model.load_state_dict(torch.load(args.weights, map_location="cpu", weights_only=True))
    model = model.cuda()
    res = evaluate(model, dicts, meta, batch_size=args.batch_size, log_every=50)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
