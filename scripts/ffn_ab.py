"""A/B: the fused FFN GEMM + GELU kernels (csrc/ffn.hip) against hipBLASLt + the separate GELU
passes, at the C2 step's FFN shapes (Swin-B 512², rgb+dte batched, B = 16: M = 16·L) and the C4
Swin-L 480x640 ones (B = 8).  Inputs rotate over buffers > 512 MB so every launch starts cold.

    python scripts/ffn_ab.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ir-ads_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from irads import native as N  # noqa: E402

SHAPES = [("c2 s0", 16 * 16384, 128, 2), ("c2 s1", 16 * 4096, 256, 2), ("c2 s2", 16 * 1024, 512, 18),
          ("c2 s3", 16 * 256, 1024, 2), ("c4 s0", 8 * 19200, 192, 2), ("c4 s1", 8 * 4800, 384, 2),
          ("c4 s2", 8 * 1200, 768, 18), ("c4 s3", 8 * 300, 1536, 2)]


def timed(fns, reps=24):
    for f in fns:
        f()
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for r in range(reps):
        fns[r % len(fns)]()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    tot = {"fwd_ref": 0., "fwd_fused": 0., "bwd_ref": 0., "bwd_fused": 0.}
    for name, M, C, blocks in SHAPES:
        nb = max(2, min(8, -(-(600 << 20) // (M * 4 * C * 2 * 3))))
        xs = [torch.randn(M, C, device=dev).bfloat16() for _ in range(nb)]
        us = [torch.empty(M, 4 * C, device=dev, dtype=torch.bfloat16) for _ in range(nb)]
        gs = [torch.empty_like(us[0]) for _ in range(nb)]
        w1 = (torch.randn(4 * C, C, device=dev) * C ** -0.5).bfloat16()
        b1 = (torch.randn(4 * C, device=dev) * 0.1).bfloat16()
        b1f = b1.float()
        w2 = (torch.randn(C, 4 * C, device=dev) * (4 * C) ** -0.5).bfloat16()
        w2t = w2.t().contiguous()

        def ref_fwd(k):
            def f():
                u = F.linear(xs[k], w1, b1)
                N.call("irads_gelu_fwd", N.ptr(u), N.ptr(gs[k]), u.numel(), N.stream())
            return f

        def fused_fwd(k):
            def f():
                N.call("irads_ffn_fc1_gelu", N.ptr(xs[k]), N.ptr(w1), N.ptr(b1f), M, C, 4 * C, N.ptr(us[k]),
                       N.ptr(gs[k]), N.stream())
            return f

        def ref_bwd(k):
            def f():
                dg = torch.mm(xs[k], w2)
                N.call("irads_gelu_bwd", N.ptr(us[k]), N.ptr(dg), N.ptr(gs[k]), dg.numel(), N.stream())
            return f

        def fused_bwd(k):
            def f():
                N.call("irads_ffn_fc2_dgrad_dgelu", N.ptr(xs[k]), N.ptr(w2t), N.ptr(us[k]), M, C, 4 * C, N.ptr(gs[k]),
                       N.stream())
            return f
        row = {"shape": name, "M": M, "C": C}
        for tag, mk in (("fwd_ref", ref_fwd), ("fwd_fused", fused_fwd), ("bwd_ref", ref_bwd),
                        ("bwd_fused", fused_bwd)):
            row[tag] = round(timed([mk(k) for k in range(nb)]), 2)
            tot[tag] += row[tag] * blocks
        flops = 2 * M * C * 4 * C
        row["fused_fwd_tflops"] = round(flops / (row["fwd_fused"] * 1e-6) / 1e12, 1)
        print(json.dumps(row), flush=True)
    print(json.dumps({k: round(v, 1) for k, v in tot.items()}))


if __name__ == "__main__":
    main()
