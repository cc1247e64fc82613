"""Window-attention kernel timing without host overhead: each (stage, shift) case captures 20
back-to-back irads_winattn_fwd (and _bwd) launches into one HIP graph and times its replays.

    python scripts/winattn_lab.py [--reps 5]

Shapes are the C2 bench step's (Swin-B at 512², rgb+dte batched: B = 16).  Bytes are SURVEY
§8(d)'s algorithmic bytes over PADDED tokens (fwd 8·Np·C, bwd 16·Np·C in bf16); the last line is
the launch-weighted average over one step's 24 launches (stage blocks 2 / 2 / 18 / 2, half shifted).
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


def graph_time(fn, n=20, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    tot = {"fwd_us": 0.0, "bwd_us": 0.0, "fwd_b": 0, "bwd_b": 0, "n": 0}
    rows = []
    for side, C, nH, blocks in STAGES:
        B, L = 16, side * side
        Hp, Wp, nW = ops._winattn_geometry(side, side)
        qkv = (torch.randn(B, L, 3 * C, device=dev) * 0.5).bfloat16()
        bias = torch.randn(3 * C, device=dev) * 0.1
        table = torch.randn(23 * 23, nH, device=dev) * 0.1
        scale = 32 ** -0.5
        quads = ops.bias_quads(table, nH, scale)
        out = torch.empty(B, L, C, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(B * nW * nH * 144, device=dev)
        gout = torch.randn(B, L, C, device=dev).bfloat16()
        gqkv = torch.empty_like(qkv)
        for shift in (0, 6):
            def fwd():
                N.call("irads_winattn_fwd", N.BF16, N.ptr(qkv), N.ptr(bias), N.ptr(table), N.ptr(quads), None, 0,
                       B, side, side, C, nH, shift, scale, N.ptr(out), N.ptr(lse), N.stream())

            def bwd():
                N.call("irads_winattn_bwd", N.BF16, N.ptr(qkv), N.ptr(bias), N.ptr(table), N.ptr(quads), None, 0,
                       B, side, side, C, nH, shift, scale, N.ptr(out), N.ptr(lse), N.ptr(gout), N.ptr(gqkv),
                       None, None, N.stream())
            fwd()
            tf = graph_time(fwd, reps=args.reps)
            tb = graph_time(bwd, reps=args.reps)
            fb, bb = B * Hp * Wp * 8 * C, B * Hp * Wp * 16 * C
            rows.append({"side": side, "C": C, "shift": shift, "fwd_us": round(tf, 2), "bwd_us": round(tb, 2),
                         "fwd_gbs": round(fb / tf / 1e3), "bwd_gbs": round(bb / tb / 1e3)})
            print(json.dumps(rows[-1]), flush=True)
            w = blocks // 2
            tot["fwd_us"] += w * tf
            tot["bwd_us"] += w * tb
            tot["fwd_b"] += w * fb
            tot["bwd_b"] += w * bb
            tot["n"] += w
    n = tot["n"]
    print(json.dumps({"step_avg": True, "launches": n, "fwd_avg_us": round(tot["fwd_us"] / n, 2),
                      "bwd_avg_us": round(tot["bwd_us"] / n, 2),
                      "fwd_frac_8TBs": round(tot["fwd_b"] / tot["fwd_us"] / 1e3 / 8000, 4),
                      "bwd_frac_8TBs": round(tot["bwd_b"] / tot["bwd_us"] / 1e3 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
