"""Per-component GPU time of the bench training step (forward + backward), each component
captured alone in a HIP graph and replayed, on the bench's shapes (Swin-B, 512², batch 8).

    python scripts/component_profile.py > gpurun_out/components.txt

Components mirror SwinTransformer.forward / CMNeXt.forward: patch embeds, MPG[i],
stage[i] (fused blocks + PatchMerging), the output norms + DeformMPG[i] (DSCF, with the
DAttn module separately), the three SegFormer heads with their resizes, and the MMST loss.
The sum is compared with the whole graphed step to show what the split misses (optimizer,
casts of parameters, gradient buffers).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ir-ads_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def leaf(t):
    if isinstance(t, torch.Tensor) and t.is_floating_point():
        return t.detach().clone().requires_grad_(True)
    return t


ONLY = None  # --only SUBSTR: time just the components whose name contains SUBSTR


def time_graph(fn, inputs, reps=20, name=""):
    """fn(*inputs) -> tensor or tuple; fwd + bwd captured once, replayed `reps` times
    (3 eager warm-up runs + 3 + reps replays execute it: 26 runs at the default)."""
    if ONLY and ONLY not in name:
        return float("nan")
    return _time_graph(fn, inputs, reps)


def _time_graph(fn, inputs, reps):
    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = fn(*inputs)
        outs = [o for o in (out if isinstance(out, (tuple, list)) else (out,)) if isinstance(o, torch.Tensor)
                and o.requires_grad]
        grads = [g for g in step.grads] if hasattr(step, "grads") else None
        if grads is None:
            step.grads = [torch.randn_like(o) * 1e-2 for o in outs]
            grads = step.grads
        torch.autograd.backward(outs, grads)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(3):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if ONLY:
        time.sleep(1.0)  # idle gap: the kernel trace after it is exactly the `reps` replays
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    if ONLY:
        time.sleep(1.0)  # closing gap: later eager work is not part of the traced replays
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True  # as bench.py: MIOpen picks its solvers by measurement
    torch.manual_seed(3407)
    model, opt, sched, loss_fn = bench.build(dev, 1, 0, 1000)
    model.train()
    rgb, dep, lbl = bench.synthetic_batch(8, 512, dev, 3407)
    bb = model.backbone
    from semseg.losses import mmst_loss
    from irads import ops
    rows = []

    # reference inputs from one real forward (autocast, as the step)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        x_rgb, hw = bb.patch_embed(rgb)
        x_dte, _ = bb.extra_patch_embed(dep)
    rows.append(("patch_embed x2", time_graph(lambda a, b: (bb.patch_embed(a)[0], bb.extra_patch_embed(b)[0]),
                                              [rgb, dep], name="patch_embed x2")))
    B = x_rgb.shape[0]
    outs, outs_rgb, outs_dte = [], [], []
    for i, stage in enumerate(bb.stages):
        mpg = bb.MPGBlocks[i]
        h, w = hw
        rows.append((f"MPG[{i}] + adds", time_graph(
            lambda a, b, m=mpg, h=h, w=w: tuple(t + f for t, f in zip((a, b), m(a, b, h, w))),
            [leaf(x_rgb), leaf(x_dte)], name=f"MPG[{i}]")))
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            f_rgb, f_dte = mpg(x_rgb, x_dte, h, w)
            x_rgb, x_dte = x_rgb + f_rgb, x_dte + f_dte
            xcat = torch.cat([x_rgb, x_dte], 0)
        rows.append((f"stage[{i}] (cat + blocks + merge)", time_graph(
            lambda a, b, st=stage, hw=hw: st.forward_pair(torch.cat([a, b], 0), hw, B)[::2],
            [leaf(x_rgb), leaf(x_dte)], name=f"stage[{i}]")))
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            xd, hw_d, xo, out_hw = stage.forward_pair(xcat, hw, B)
        xo_r, xo_d = xo[:B].contiguous(), xo[B:].contiguous()
        rows.append((f"outputs[{i}] (3 LN + DeformMPG)", time_graph(
            lambda a, b, i=i, ohw=out_hw: bb._outputs(i, a, b, ohw), [leaf(xo_r), leaf(xo_d)],
            name=f"outputs[{i}]")))
        # the DAttn module inside DeformMPG alone
        dm = bb.DeformMPGBlocks[i]
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            nr = getattr(bb, f"norm{i}")(xo_r)
            nd = getattr(bb, f"extra_norm{i}")(xo_d)
            xr = dm.D_fc1(nr)
            xdd = dm.D_fc2(nd)
            Bq, Nq, c = xr.shape
            xr = xr.reshape(Bq, *out_hw, c).permute(0, 3, 1, 2).contiguous()
            xdd = xdd.reshape(Bq, *out_hw, c).permute(0, 3, 1, 2).contiguous()
        rows.append((f"  of which DAttn[{i}]", time_graph(lambda a, b, m=dm.deform_atten: m(a, b),
                                                          [leaf(xr), leaf(xdd)], name=f"DAttn[{i}]")))
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            o, orgb, odte = bb._outputs(i, xo_r, xo_d, out_hw)
        outs.append(o)
        outs_rgb.append(orgb)
        outs_dte.append(odte)
        x_rgb, x_dte, hw = xd[:B], xd[B:], hw_d
    size = rgb.shape[2:]
    for name, head, feats in (("decode_head", model.decode_head, outs), ("decode_head_rgb", model.decode_head_rgb,
                              outs_rgb), ("decode_head_dte", model.decode_head_dte, outs_dte)):
        rows.append((f"{name} + resize", time_graph(lambda *f, hd=head: ops.resize(hd(list(f)), size),
                                                    [leaf(t) for t in feats], name=name)))
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        lg = ops.resize(model.decode_head(outs), size)
    rows.append(("MMST loss", time_graph(lambda a, b, c: mmst_loss(loss_fn, a, b, c, lbl),
                                         [leaf(lg), leaf(lg.clone()), leaf(lg.clone())], name="loss")))
    total = sum(t for n, t in rows if not n.startswith("  ") and t == t)
    for n, t in rows:
        print(f"{t:8.3f} ms  {n}")
    print(f"{total:8.3f} ms  sum of components (fwd+bwd)")


if __name__ == "__main__":
    if "--only" in sys.argv:
        ONLY = sys.argv[sys.argv.index("--only") + 1]
    main()
