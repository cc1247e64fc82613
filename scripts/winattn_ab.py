"""A/B of the bf16 window-attention forward kernels at the C2 step's 8 launch shapes (Swin-B 512²,
rgb+dte batched: B = 16), in the cache state of the training step: every launch reads its own
qkv buffer (NBUF rotating buffers per shape, > 2x the 256 MB Infinity Cache in total), K launches
back to back inside one event pair behind a GPU spin.  Also checks the two variants bit for bit.

    python scripts/winattn_ab.py [--reps 24]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ir-ads_amd"))

import torch  # noqa: E402

from irads import native as N, ops  # noqa: E402

STAGES = ((128, 128, 4, 2), (64, 256, 8, 2), (32, 512, 16, 18), (16, 1024, 32, 2))  # side, C, heads, blocks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=24)
    ap.add_argument("--variants", default="0,1")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = N.load()
    torch.manual_seed(0)
    variants = [int(v) for v in args.variants.split(",")]
    tot = {v: [0.0, 0] for v in variants}
    rows = []
    for side, C, nH, blocks in STAGES:
        B, L = 16, side * side
        Hp, Wp, nW = ops._winattn_geometry(side, side)
        per = B * L * 3 * C * 2
        nbuf = max(2, min(args.reps, -(-(600 << 20) // per)))
        bufs = [(torch.randn(B, L, 3 * C, device=dev) * 0.5).bfloat16() for _ in range(nbuf)]
        bias = torch.randn(3 * C, device=dev) * 0.1
        table = torch.randn(23 * 23, nH, device=dev) * 0.1
        nbytes = B * Hp * Wp * 4 * C * 2
        for shift in (0, 6):
            outs = {}
            for v in variants:
                lib.irads_winattn_fwd_variant(v)
                outs[v] = ops.winattn_fwd(bufs[0], bias, table, None, side, side, nH, shift, 32 ** -0.5)
                for k in range(nbuf):  # warm (kernel load, quads cache)
                    ops.winattn_fwd(bufs[k], bias, table, None, side, side, nH, shift, 32 ** -0.5)
                torch.cuda.synchronize()
                torch.cuda._sleep(200_000)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for r in range(args.reps):
                    ops.winattn_fwd(bufs[r % nbuf], bias, table, None, side, side, nH, shift, 32 ** -0.5)
                b.record()
                torch.cuda.synchronize()
                us = a.elapsed_time(b) * 1e3 / args.reps
                w = blocks // 2  # launches of this (shape, shift) per step
                tot[v][0] += us * w
                tot[v][1] += nbytes * w
                rows.append({"side": side, "C": C, "shift": shift, "variant": v, "us": round(us, 2),
                             "frac_of_8TBs": round(nbytes / (us * 1e-6) / 8e12, 4), "nbuf": nbuf})
                print(json.dumps(rows[-1]), flush=True)
            if len(variants) > 1:
                same = all(torch.equal(outs[variants[0]][i], outs[v][i]) for v in variants[1:] for i in (0, 1))
                print(f"side={side} shift={shift}: variants bit-identical: {same}", flush=True)
                assert same
    for v in variants:
        us, nb = tot[v]
        print(json.dumps({"variant": v, "step_fwd_us": round(us, 1), "frac_of_8TBs": round(nb / (us * 1e-6) / 8e12, 4)}))


if __name__ == "__main__":
    main()
