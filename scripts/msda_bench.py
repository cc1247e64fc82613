"""MSDeformAttn kernel lines of bench.py alone (C5 DINO encoder / decoder shapes).

    python scripts/msda_bench.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    for k, v in bench.msda_rooflines(torch.device("cuda:0")).items():
        print(k, json.dumps(v))
