"""Diagnostic (GPU box): the product's fp32 DeformMPG blocks against the fp64 oracle ON THE
PRODUCT'S OWN INPUTS.  Runs one fp32 training step of a train fixture's model, captures every
DeformMPGBlock's inputs and upstream gradient, then replays each block on the CPU oracle in fp64
and in fp32 with those exact tensors and reports the relative L2 of every parameter and input
gradient.  Separates a block's own arithmetic from sensitivity to its inputs.

    python scripts/diag_dmpg.py c4_swinl_480x640 [block ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ir-ads_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402


def rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


def main():
    tag = sys.argv[1]
    blocks = [int(b) for b in sys.argv[2:]] or [0, 1, 2, 3]
    import test_gpu_train_parity as T
    import irads_ref as R
    from golden_util import Fixture
    from semseg.losses import get_loss
    fx = Fixture(f"train_{tag}.npz")
    model, batch = T._build(fx)
    cap = {}

    def fwd_hook(i):
        def h(mod, args, out):
            cap[i] = {"args": [a.detach().clone() if torch.is_tensor(a) else a for a in args]}
            out.register_hook(lambda g: cap[i].__setitem__("gout", g.detach().clone()))
        return h
    hs = [model.backbone.DeformMPGBlocks[i].register_forward_hook(fwd_hook(i)) for i in blocks]
    amp = bool(os.environ.get("DIAG_AMP"))
    T._fwd_bwd(model, get_loss("CrossEntropy", 255), batch, amp=amp)
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    if amp:  # bf16: the block's fast path vs its module path vs fp32, on the captured inputs
        from irads import ops
        for i in blocks:
            blk = model.backbone.DeformMPGBlocks[i]
            args, gout = cap[i]["args"], cap[i]["gout"]
            res = {}
            for mode in ("fast", "module", "fp32"):
                orig = ops.dattn_offset_ok
                if mode != "fast":
                    ops.dattn_offset_ok = lambda *a, **k: False
                try:
                    for p in blk.parameters():
                        p.grad = None
                    a = (args[0].float() if mode == "fp32" else args[0]).clone().requires_grad_()
                    b = (args[1].float() if mode == "fp32" else args[1]).clone().requires_grad_()
                    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode != "fp32"):
                        o = blk(a, b, *args[2:])
                    o.backward(gout.to(o.dtype))
                finally:
                    ops.dattn_offset_ok = orig
                res[mode] = {n: p.grad.detach().double().cpu() for n, p in blk.named_parameters() if p.grad is not None}
            print(f"block {i} (bf16 fast / module vs fp32 on the captured inputs):", flush=True)
            rows = sorted(((rel(res["fast"][n], res["fp32"][n]), rel(res["module"][n], res["fp32"][n]), n)
                           for n in res["fp32"] if float(res["fp32"][n].norm()) > 0), reverse=True)
            for r in rows[:12]:
                print("   fast %.2e  module %.2e  %s" % r, flush=True)
            for r in rows:
                if "get_sample_weight" in r[2]:
                    print("   fast %.2e  module %.2e  %s" % r, flush=True)
        return
    report = {}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    if os.environ.get("DIAG_SAVE"):
        for i in blocks:
            torch.save({"x_rgb": cap[i]["args"][0].cpu(), "x_dte": cap[i]["args"][1].cpu(), "gout": cap[i]["gout"].cpu()},
                       os.path.join(ROOT, "gpurun_out", f"dmpg_io_{tag}_{i}.pt"))
    for i in blocks:
        blk = model.backbone.DeformMPGBlocks[i]
        bb = model.backbone
        # the product block's own parameter gradients came only from this block's inputs and gout;
        # recompute them on the product (fresh) to isolate the block
        args = cap[i]["args"]
        xr = args[0].clone().requires_grad_()
        xd = args[1].clone().requires_grad_()
        for p in blk.parameters():
            p.grad = None
        out = blk(xr, xd, *args[2:])
        out.backward(cap[i]["gout"])
        prod = {n: p.grad.detach().cpu() for n, p in blk.named_parameters() if p.grad is not None}
        prod["in.x_rgb"], prod["in.x_dte"] = xr.grad.cpu(), xd.grad.cpu()
        prod["out"] = out.detach().cpu()
        res = {}
        for dt in (torch.float64, torch.float32):
            ref = R.DeformMPGBlock(blk.D_fc1.in_features, blk.deform_atten.stride, blk.deform_atten.n_groups,
                                   blk.deform_atten.n_heads, 0.0, i, 1 / 8)
            sd = {k: v.detach().cpu() for k, v in blk.state_dict().items()}
            ref.load_state_dict(sd)
            ref = ref.to(dt)
            ref.train()
            a = xr.detach().cpu().to(dt).requires_grad_()
            b = xd.detach().cpu().to(dt).requires_grad_()
            o = ref(a, b, *args[2:])
            o.backward(cap[i]["gout"].cpu().to(dt))
            g = {n: p.grad.detach() for n, p in ref.named_parameters() if p.grad is not None}
            g["in.x_rgb"], g["in.x_dte"], g["out"] = a.grad, b.grad, o.detach()
            res[dt] = g
        rows = {}
        for n in prod:
            if n not in res[torch.float64]:
                continue
            rows[n] = {"prod32_vs_ref64": rel(prod[n], res[torch.float64][n]),
                       "ref32_vs_ref64": rel(res[torch.float32][n], res[torch.float64][n])}
        report[f"DeformMPGBlocks.{i}"] = rows
        worst = sorted(((v["prod32_vs_ref64"], v["ref32_vs_ref64"], n) for n, v in rows.items()), reverse=True)[:8]
        print(f"block {i}:", flush=True)
        for w in worst:
            print("   prod32 %.2e  ref32 %.2e  %s" % w, flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"diag_dmpg_{tag}.json"), "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
