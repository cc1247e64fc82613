"""Workgroup timelines of the stamped launches of one bench step (IRADS_STAMP_DUMP=<file>.npz bench.py).

    python scripts/stamp_timeline.py gpurun_out/stamps.npz [--name winattn_fwd]

Per launch: workgroups, span, workgroup duration (min / median / max), the start-time spread (how
long the dispatcher takes to start every workgroup) and the time the last `tail` fraction of the
span runs with fewer than half of the peak concurrency (the round tail)."""
import sys

import numpy as np


def main():
    d = np.load(sys.argv[1])
    name = sys.argv[sys.argv.index("--name") + 1] if "--name" in sys.argv else "winattn_fwd"
    khz = float(d["khz"])
    us = 1e3 / khz  # microseconds per tick
    for i, (n, nb) in enumerate(zip(d["names"], d["bytes"])):
        if n != name:
            continue
        r = d["regions"][i]
        ok = (r[:, 0] > 0) & (r[:, 1] > 0)
        st, en = r[ok, 0].astype(np.int64), r[ok, 1].astype(np.int64)
        if not len(st):
            continue
        t0 = st.min()
        span = (en.max() - t0) * us
        dur = (en - st) * us
        # concurrency over time (resident workgroups)
        ev = np.concatenate([np.stack([st - t0, np.ones_like(st)], 1), np.stack([en - t0, -np.ones_like(en)], 1)])
        ev = ev[np.argsort(ev[:, 0], kind="stable")]
        conc = np.cumsum(ev[:, 1])
        peak = conc.max()
        times = ev[:, 0] * us
        low = 0.0
        for k in range(len(ev) - 1):
            if conc[k] < peak / 2:
                low += times[k + 1] - times[k]
        print(f"slot {i:3d} wg {ok.sum():5d} bytes {nb / 1e6:6.1f} MB span {span:6.1f} us  "
              f"wg dur min/med/max {dur.min():5.1f}/{np.median(dur):5.1f}/{dur.max():5.1f} us  "
              f"start spread {(st.max() - t0) * us:5.1f} us  peak resident {peak:5d}  "
              f"below half-peak {low:5.1f} us  -> {nb / span / 1e3 / 8000:.3f} of 8 TB/s")


if __name__ == "__main__":
    main()
