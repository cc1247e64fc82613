"""The FFN's fused GEMMs on the 256 x 256 tiling (fc1 + GELU, fc2 dX + GELU') at the C2 stage shapes:
median time per call, GELU by table (default) or by formula (IRADS_GEMM_GELU_TABLE=0, read once per
process: run the script once each way on one box).

    python scripts/gelu_table_ab.py
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

import torch  # noqa: E402

from irads import native as N  # noqa: E402


def timed(fn, reps=10):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    mode = "formula" if os.environ.get("IRADS_GEMM_GELU_TABLE") == "0" else "table"
    total = 0.0
    for C, M, blocks in ((128, 262144, 2), (256, 65536, 2), (512, 16384, 18), (1024, 4096, 2)):
        C4 = 4 * C
        A = torch.randn(M, C, device=dev).bfloat16()
        W1 = (torch.randn(C4, C, device=dev) * C ** -0.5).bfloat16()
        b32 = (torch.randn(C4, device=dev) * 0.1).bfloat16().float()
        u, g = (torch.empty(M, C4, device=dev, dtype=torch.bfloat16) for _ in range(2))
        dF = torch.randn(M, C, device=dev).bfloat16()
        W2t = (torch.randn(C4, C, device=dev) * C4 ** -0.5).bfloat16()  # (4C, C): fc2's W transposed
        U = (torch.randn(M, C4, device=dev) * 1.5).bfloat16()
        du = torch.empty(M, C4, device=dev, dtype=torch.bfloat16)

        def fwd():
            N.call("irads_gemm_nt_variant", 4, 1, N.ptr(A), A.stride(0), N.ptr(W1), W1.stride(0), N.ptr(b32), None, 0,
                   N.ptr(u), N.ptr(g), u.stride(0), M, C4, C, N.stream())

        def bwd():
            N.call("irads_gemm_nt_variant", 4, 2, N.ptr(dF), dF.stride(0), N.ptr(W2t), W2t.stride(0), None, N.ptr(U),
                   U.stride(0), N.ptr(du), None, du.stride(0), M, C4, C, N.stream())
        fwd(), bwd()
        tf = statistics.median(timed(fwd) for _ in range(5))
        tb = statistics.median(timed(bwd) for _ in range(5))
        total += (tf + tb) * blocks
        print(json.dumps({"mode": mode, "C": C, "M": M, "fwd_gelu_us": round(tf, 2), "bwd_dgelu_us": round(tb, 2)}),
              flush=True)
    print(json.dumps({"mode": mode, "ffn_fused_ms_per_step": round(total / 1e3, 3)}))


if __name__ == "__main__":
    main()
