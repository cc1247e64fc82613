"""Produce the hipBLASLt selection table for the bench step (PyTorch TunableOp), on an MI355X.

    python scripts/tune_gemms.py --out gpurun_out/tunableop_mi355x0.csv [--workload c4]
    python scripts/tune_gemms.py --out gpurun_out/tunableop_c4.csv --merge-into ir-ads_amd/irads/tuned/tunableop_mi355x0.csv
then copy the file to ir-ads_amd/irads/tuned/tunableop_mi355x0.csv (read by
irads.gemm_tuning.use_tuned_gemms, which bench.py calls).  Runs eager training steps of the
bench configuration with tuning on, so every GEMM shape of the step is benchmarked once.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ir-ads_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from irads.gemm_tuning import start_tuning  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--max-ms", type=int, default=30)
    ap.add_argument("--workload", default="c2", help="bench.py workload whose step is tuned (c2, c3, c4)")
    ap.add_argument("--merge-into", default=None,
                    help="no tuning: rewrite this table as its entries overlaid by --out's (a finished run's)")
    a = ap.parse_args()
    if a.merge_into:
        merge_tables(a.out, a.merge_into)
        return
    start_tuning(a.out, a.max_ms)
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    wl = dict(bench.WORKLOADS[a.workload])
    model, opt, sched, loss_fn = bench.build(dev, 1, 0, 1000, wl=wl)
    model.train()
    batch = bench.synthetic_batch(wl["batch"], wl["hw"], dev, 3407, wl["n_cls"])
    for i in range(a.steps):
        bench.train_step(model, opt, sched, loss_fn, batch)
        torch.cuda.synchronize()
        print(f"tuning step {i} done, {len(torch.cuda.tunable.get_results())} GEMM results", flush=True)
    print("TunableOp writes", a.out, "at exit; merge it over a shipped table with", flush=True)
    print(f"    python scripts/tune_gemms.py --merge-into <table> --out {a.out}", flush=True)


def merge_tables(new, old):
    """Rewrite `old` as its entries overlaid by `new`'s (keys: op and shape columns), validators from `new`."""
    def rows(path):
        with open(path) as f:
            return [l.rstrip("\n") for l in f if l.strip()]
    import glob
    new = sorted(glob.glob(new.replace(".csv", "*.csv")))[0]
    nl, ol = rows(new), rows(old)
    val = [l for l in nl if l.startswith("Validator")]
    ent = {tuple(l.split(",")[:2]): l for l in ol if not l.startswith("Validator")}
    ent.update({tuple(l.split(",")[:2]): l for l in nl if not l.startswith("Validator")})
    with open(old, "w") as f:
        f.write("\n".join(val + list(ent.values())) + "\n")
    print("merged", len(ent), "entries into", old)


if __name__ == "__main__":
    main()
