"""How the three clocks bench.py's roofline could use compare on ONE kernel shape.

    rocprofv3 --kernel-trace --stats -d gpurun_out/tc -o tc -- python3 scripts/timing_check.py

The C2 step's stage-2 window-attention forward (Swin-B, 32x32 tokens, C = 512, 16 heads, rgb + dte
batched: B = 16), launched `reps` times back to back over 8 distinct input sets (no launch finds
its inputs in the caches), timed three ways:
  * one HIP event pair around all launches (per-launch = total / reps: includes every inter-kernel
    gap, i.e. an upper bound of the kernels' own time);
  * in-kernel wall-clock stamps per launch (ops.STAMPS: first workgroup start -> last workgroup end);
  * the rocprofv3 kernel trace of this same process (read from its output afterwards).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ir-ads_amd"))

import torch  # noqa: E402

from irads import ops  # noqa: E402


def main(reps=200, sets=8):
    dev = torch.device("cuda", 0)
    side, C, nH, B = 32, 512, 16, 16
    L = side * side
    g = torch.Generator(device="cpu").manual_seed(0)
    qkvs = [(torch.randn(B, L, 3 * C, generator=g) * 0.5).bfloat16().to(dev) for _ in range(sets)]
    bias = torch.randn(3 * C, generator=g).to(dev) * 0.1
    table = torch.randn(23 * 23, nH, generator=g).to(dev) * 0.1
    scale = 32 ** -0.5

    def launch(i):
        ops.winattn_fwd(qkvs[i % sets], bias, table, None, side, side, nH, 0, scale)
    for i in range(2 * sets):
        launch(i)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(reps):
        launch(i)
    b.record()
    torch.cuda.synchronize()
    ev_us = a.elapsed_time(b) * 1e3 / reps
    ops.STAMPS.arm(("winattn_fwd",), dev)
    for i in range(min(reps, ops.STAMPS.CAPACITY)):
        launch(i)
    ops.STAMPS.disarm()
    sp = ops.STAMPS.read()["winattn_fwd"]
    st_us = 1e3 * sp["total_ms"] / sp["launches"]
    nbytes = B * (-(-side // 12) * 12) ** 2 * 4 * C * 2  # 8·Np·C bytes (bf16)
    print(json.dumps({"shape": f"winattn_fwd bf16 B={B} {side}x{side} C={C} heads={nH} shift=0",
                      "event_pair_us_per_launch": round(ev_us, 2), "stamp_span_us": round(st_us, 2),
                      "stamp_launches": sp["launches"], "algorithmic_bytes": nbytes,
                      "frac_events": round(nbytes / ev_us / 1e3 / 8000.0, 4),
                      "frac_stamps": round(nbytes / st_us / 1e3 / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
