"""Produce the hipBLASLt selection table for the bench step (PyTorch TunableOp), on an MI355X.

    python scripts/tune_gemms.py --out gpurun_out/tunableop_mi355x0.csv
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
    a = ap.parse_args()
    start_tuning(a.out, a.max_ms)
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    model, opt, sched, loss_fn = bench.build(dev, 1, 0, 1000)
    model.train()
    batch = bench.synthetic_batch(8, 512, dev, 3407)
    for i in range(a.steps):
        bench.train_step(model, opt, sched, loss_fn, batch)
        torch.cuda.synchronize()
        print(f"tuning step {i} done, {len(torch.cuda.tunable.get_results())} GEMM results", flush=True)
    print("TunableOp writes", a.out, "at exit")


if __name__ == "__main__":
    main()
