"""Device time of every aten op (the torch "glue" between the HIP kernels) in one eager bench step,
by issuing site: a TorchDispatchMode brackets each op with HIP events and attributes it to the
Python frame inside the package (forward) or the autograd node (backward), as cast_audit.py does.
GEMMs / convolutions are aten ops too and are listed; the irads kernels are not (they are not
dispatched through aten).

    python scripts/glue_profile.py [--batch 8] [--top 50]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd"), os.path.join(ROOT, "scripts")]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402
from cast_audit import NO_KERNEL, site  # noqa: E402


class Timer(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ev = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        short = str(func).replace("aten.", "").replace(".default", "")
        if short in NO_KERNEL:
            return func(*args, **(kwargs or {}))
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = func(*args, **(kwargs or {}))
        b.record()
        t = out if torch.is_tensor(out) else (args[0] if args and torch.is_tensor(args[0]) else None)
        shape = tuple(t.shape) if t is not None else ()
        dt = str(t.dtype).replace("torch.", "") if t is not None else ""
        self.ev.append((short, site(), shape, dt, a, b))
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--top", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(3407)
    model, opt, sched, loss_fn = bench.build(dev, 1, 0, 1000)
    model.train()
    batch = bench.synthetic_batch(a.batch, 512, dev, 3407)
    for _ in range(2):
        bench.train_step(model, opt, sched, loss_fn, batch)
    torch.cuda.synchronize()
    tm = Timer()
    with tm:
        bench.train_step(model, opt, sched, loss_fn, batch)
    torch.cuda.synchronize()
    by_site = collections.defaultdict(lambda: [0, 0.0, collections.Counter()])
    total = 0.0
    for op, st, shape, dt, ea, eb in tm.ev:
        ms = ea.elapsed_time(eb)
        r = by_site[(op, st, dt)]
        r[0] += 1
        r[1] += ms
        r[2][shape] += 1
        total += ms
    print(f"aten ops: {len(tm.ev)} calls, {total:.3f} ms of event time (includes launch gaps)")
    for (op, st, dt), (n, ms, shapes) in sorted(by_site.items(), key=lambda kv: -kv[1][1])[:a.top]:
        sh = ", ".join(f"{s}x{c}" for s, c in shapes.most_common(2))
        print(f"{ms * 1e3:8.1f} us {n:4d}x  {op:18s} {dt:9s} {st[:95]:95s} {sh[:80]}")


if __name__ == "__main__":
    main()
