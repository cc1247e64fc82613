"""The C5 vCLR DINO-R50 detector training-step line (bench.py --detector's), on its own:

    python scripts/dino_detector_bench.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    # MIOpen's benchmark search for every ResNet-50 shape at 800x1333 takes minutes on its first step;
    # its immediate-mode solvers are used instead (IRADS_DET_BENCHMARK=1 restores the search)
    torch.backends.cudnn.benchmark = os.environ.get("IRADS_DET_BENCHMARK") == "1"
    import threading
    import time
    t0 = time.time()

    def beat():  # a line a minute, so a long first step is not taken for a hang
        while True:
            time.sleep(60)
            print(f"[detector] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    line = bench.dino_detector_line(torch.device("cuda:0"))
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join("gpurun_out", "dino_detector_c5.json")
    with open(out, "w") as fh:
        json.dump(line, fh, indent=1)
    print(json.dumps(line))


if __name__ == "__main__":
    main()
