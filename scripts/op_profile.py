"""Operator-level profile of the bench training step (torch.profiler, GPU time per aten op
and input shapes), to attribute the non-irads kernels to the model code that issues them.

    python scripts/op_profile.py [--steps 3] [--rows 60] > gpurun_out/ops.txt
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ir-ads_amd"))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--rows", type=int, default=60)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--stacks", default=None, help="comma-separated aten ops: print their Python call stacks")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(3407)
    model, opt, sched, loss_fn = bench.build(dev, 1, 0, 1000)
    model.train()
    batch = bench.synthetic_batch(a.batch, 512, dev, 3407)
    for _ in range(3):
        bench.train_step(model, opt, sched, loss_fn, batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=a.stacks is not None) as prof:
        for _ in range(a.steps):
            bench.train_step(model, opt, sched, loss_fn, batch)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=50,
                   max_shapes_column_width=70))
    # aten ops with full shapes: GPU time per step and achieved rate for the GEMMs
    rows = []
    for e in ka:
        if not e.key.startswith("aten::") or e.self_device_time_total <= 0:
            continue
        rows.append((e.self_device_time_total / a.steps, e.count / a.steps, e.key, str(e.input_shapes)))
    rows.sort(reverse=True)
    print("\n# aten ops by GPU time per step (us), calls per step, shapes")
    for us, n, k, shp in rows[:a.rows]:
        extra = ""
        try:
            sh = eval(shp)
            if k in ("aten::mm",) and len(sh[0]) == 2:
                M, K = sh[0]; N_ = sh[1][1]
                extra = f"  {2 * M * K * N_ * n / us / 1e6:8.1f} TF/s"
            if k in ("aten::addmm",) and len(sh[1]) == 2:
                M, K = sh[1]; N_ = sh[2][1]
                extra = f"  {2 * M * K * N_ * n / us / 1e6:8.1f} TF/s"
        except Exception:
            pass
        print(f"{us:9.1f} {n:6.1f}  {k:34s} {shp[:150]}{extra}")
    if a.stacks:
        want = set(a.stacks.split(","))
        print("\n# call stacks (GPU us per step, calls per step)")
        for e in sorted(prof.key_averages(group_by_stack_n=6), key=lambda e: -e.self_device_time_total):
            if e.key in want and e.self_device_time_total > 0:
                print(f"{e.self_device_time_total / a.steps:9.1f} {e.count / a.steps:6.1f} {e.key}")
                for fr in e.stack:
                    print("          ", fr)
    # backward nodes: GPU time (self + children) per step, to attribute fills / casts / adds
    ka2 = prof.key_averages()
    rows = [(e.device_time_total / a.steps, e.count / a.steps, e.key) for e in ka2
            if e.key.startswith("autograd::engine::evaluate_function") and e.device_time_total > 0]
    rows.sort(reverse=True)
    print("\n# autograd nodes by GPU time per step (us, incl. children), calls per step")
    for us, n, k in rows[:a.rows]:
        print(f"{us:9.1f} {n:6.1f}  {k[len('autograd::engine::evaluate_function: '):]}")


if __name__ == "__main__":
    main()
