"""Every library GEMM (aten mm / addmm / linear / bmm) of one eager C2 training step with its shape,
the calling module and its time (HIP events around the op): which shapes still run on hipBLASLt.

    python scripts/gemm_shapes_step.py > gpurun_out/gemm_shapes_step.json
"""
import collections
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402

OPS = {"aten.mm.default", "aten.addmm.default", "aten.bmm.default", "aten._addmm_activation.default"}


class Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.defaultdict(lambda: [0, 0.0])

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if name not in OPS:
            return func(*args, **(kwargs or {}))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = func(*args, **(kwargs or {}))
        b.record()
        b.synchronize()
        shapes = tuple(tuple(t.shape) for t in args if torch.is_tensor(t))
        st = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in traceback.extract_stack()[-12:-2]
              if "ir-ads_amd" in f.filename]
        key = (name, shapes, str(args[0].dtype) if torch.is_tensor(args[0]) else "", st[-1] if st else "?")
        self.rows[key][0] += 1
        self.rows[key][1] += a.elapsed_time(b)
        return out


def main():
    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS["c2"]
    model, opt, sched, loss_fn = bench.build(dev, 1, 0, 100, wl=wl)
    batch = bench.synthetic_batch(wl["batch"], wl["hw"], dev, 0, wl["n_cls"])
    for _ in range(2):
        bench.train_step(model, opt, sched, loss_fn, batch)
    torch.cuda.synchronize()
    rec = Rec()
    with rec:
        bench.fwd_bwd(model, loss_fn, batch)
    torch.cuda.synchronize()
    out = [{"op": k[0], "shapes": k[1], "dtype": k[2], "site": k[3], "n": v[0], "ms": round(v[1], 4)}
           for k, v in sorted(rec.rows.items(), key=lambda kv: -kv[1][1])]
    print(json.dumps({"total_ms": round(sum(r["ms"] for r in out), 3), "gemms": out}, indent=1))


if __name__ == "__main__":
    main()
