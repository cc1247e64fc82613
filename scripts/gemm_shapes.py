"""The Swin-B trunk's library GEMMs at the C2 step's shapes (rgb + dte batched, B = 8, 512²), in
isolation, with the shipped TunableOp table: time per call, TFLOP/s, and the fraction of the
shape's own bound max(flops / 2.5 PF, bytes / 8 TB/s).  Forward: y = x Wᵀ + b (F.linear under
the same bf16 operands autocast produces); backward: dX = dY W (the trunk is frozen: no dW).

    python scripts/gemm_shapes.py [--untuned]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

STAGES = ((128, 262144, 2), (256, 65536, 2), (512, 16384, 18), (1024, 4096, 2))  # C, tokens, blocks
PEAK_F, PEAK_B = 2.5e15, 8e12


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    torch.cuda._sleep(100_000)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    from irads.gemm_tuning import use_tuned_gemms
    print("tuned table:", use_tuned_gemms() if "--untuned" not in sys.argv else "off (hipBLASLt heuristic)")
    dev = torch.device("cuda:0")
    tot = {"us": 0.0, "bound_us": 0.0}
    for C, M, blocks in STAGES:
        for op, K, N in (("qkv", C, 3 * C), ("proj", C, C), ("fc1", C, 4 * C), ("fc2", 4 * C, C)):
            x = torch.randn(M, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
            bias = torch.randn(N, device=dev).bfloat16()
            dy = torch.randn(M, N, device=dev).bfloat16()
            flops = 2.0 * M * K * N
            for d, fn, nbytes in (("fwd", lambda: F.linear(x, w, bias), 2 * (M * K + K * N + M * N)),
                                  ("bwd", lambda: torch.mm(dy, w), 2 * (M * N + K * N + M * K))):
                us = timed(fn)
                bound = max(flops / PEAK_F, nbytes / PEAK_B) * 1e6
                tot["us"] += us * blocks
                tot["bound_us"] += bound * blocks
                print(json.dumps({"C": C, "M": M, "op": op, "dir": d, "K": K, "N": N, "us": round(us, 1),
                                  "tflops": round(flops / us / 1e6, 1), "frac_of_bound": round(bound / us, 3),
                                  "per_step_us": round(us * blocks, 1)}), flush=True)
            del x, w, bias, dy
    print(json.dumps({"trunk_gemm_ms_per_step": round(tot["us"] / 1e3, 3),
                      "bound_ms_per_step": round(tot["bound_us"] / 1e3, 3)}))


if __name__ == "__main__":
    main()
