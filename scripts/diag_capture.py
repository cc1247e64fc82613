"""Diagnose a HIP-graph capture crash of the CMNeXt training step: each variant runs in its own
subprocess (python scripts/diag_capture.py VARIANT), the driver loop reports which crash."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ir-ads_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

VARIANTS = ["det_noeager", "det_droppath", "det_adapterdrop", "det_head_drop", "rand_nomask", "det_b4"]


def run(variant):
    import torch
    from fill import fill_module
    from semseg.models import CMNeXt
    from semseg.losses import get_loss, mmst_loss
    from train_fixture import adapter_trainable, deterministic_train_mode, train_inputs
    dev = torch.device("cuda", 0)
    B = 4 if variant == "det_b4" else 2
    model = CMNeXt("SwinTransformer-B", 40, ["img", "depth"])
    fill_module(model, seed=41)
    model = model.to(dev)
    for n, p in model.named_parameters():
        p.requires_grad_(adapter_trainable(n))
    deterministic_train_mode(model)
    if variant == "det_droppath":
        for m in model.modules():
            if type(m).__name__ == "DropPath":
                m.p = 0.1
    if variant == "det_adapterdrop":
        for m in model.modules():
            if type(m).__name__ == "Adapter":
                m.training = True
    if variant == "det_head_drop":
        for m in model.modules():
            if isinstance(m, torch.nn.Dropout2d):
                m.p = 0.1
    if variant == "rand_nomask":
        model.train()
        model.backbone.training = False
    rgb, dep, lbl = [torch.from_numpy(a).to(dev) for a in train_inputs(B, 512, 512, 40, 200)]
    loss_fn = get_loss("CrossEntropy", 255)
    params = [p for p in model.parameters() if p.requires_grad]

    def fb():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y, yr, yd = model([rgb, dep])
            loss = mmst_loss(loss_fn, y, yr, yd, lbl)
        loss.backward()
        return loss
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            for p in params:
                p.grad = None
            fb()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    for p in params:
        p.grad = None
    g = torch.cuda.CUDAGraph()
    print(variant, "capturing", flush=True)
    with torch.cuda.graph(g):
        loss = fb()
    print(variant, "captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(variant, "ok loss", float(loss), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
        sys.exit(0)
    for v in VARIANTS:
        r = subprocess.run([sys.executable, "-u", __file__, v], capture_output=True, text=True, timeout=180)
        tail = (r.stdout + r.stderr).strip().splitlines()[-3:]
        print(f"{v}: rc={r.returncode} :: " + " | ".join(tail), flush=True)
