"""The vCLR DINO transformer line of bench.py on its own (for profiling):
    python scripts/dino_bench.py            # prints the msda lines + dino_transformer_c5 as JSON
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    k = bench.msda_rooflines(dev)
    k["dino_transformer_c5"] = bench.dino_stack_line(dev, k, reps=int(os.environ.get("DINO_REPS", "5")))
    print(json.dumps(k))
