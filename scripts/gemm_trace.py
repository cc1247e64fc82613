"""Where irads_gemm_nt's time goes: every workgroup's wall_clock64() stamps (100 MHz) at entry, after
each k-step's barrier, after the main loop and at exit (irads_gemm_nt_trace), summarised per shape:
first-stage latency, k-step time, epilogue, workgroup lifetime and the launch's span.

    python scripts/gemm_trace.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from irads import native as N  # noqa: E402

SHAPES = (("s2_proj", 16384, 512, 512), ("s2_fc1", 16384, 2048, 512), ("s2_fc2", 16384, 512, 2048),
          ("s0_fc1", 262144, 512, 128), ("s3_fc2", 4096, 1024, 4096), ("s2_qkv", 16384, 1536, 512))


def main():
    dev = torch.device("cuda:0")
    for name, M, Nn, K in SHAPES:
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(Nn, K, device=dev) * K ** -0.5).bfloat16()
        bias = torch.zeros(Nn, device=dev)
        C = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        nk = K // 64
        variant = int(os.environ.get("GEMM_VARIANT", "2"))
        bmt = 256 if variant in (0, 1, 4) else 128
        bnt = 256 if variant == 4 else 128
        nwg = (M + bmt - 1) // bmt * (Nn // bnt)
        tr = torch.zeros(nwg * (nk + 3), dtype=torch.int64, device=dev)
        args = (variant, N.ptr(A), A.stride(0), N.ptr(W), W.stride(0), N.ptr(bias), N.ptr(C), C.stride(0), M, Nn, K,
                N.ptr(tr), N.stream())
        for _ in range(3):
            N.call("irads_gemm_nt_trace", *args)
        torch.cuda.synchronize()
        t = tr.view(nwg, nk + 3).cpu().numpy().astype(np.float64) * 10.0  # ns
        t0 = t[:, 0].min()
        t -= t0
        life = t[:, -1] - t[:, 0]
        first = t[:, 1] - t[:, 0]
        steps = np.diff(t[:, 1:nk + 1], axis=1) if nk > 1 else np.zeros((nwg, 1))
        last = t[:, nk + 1] - t[:, nk]          # last k-step's compute + the epilogue barrier
        epi = t[:, -1] - t[:, nk + 1]
        ref = (A.float() @ W.float().t()).bfloat16()
        err = float((C.float() - ref.float()).norm() / ref.float().norm())
        print(json.dumps({
            "shape": name, "variant": variant, "M": M, "N": Nn, "K": K, "wg": nwg, "rel_err": round(err, 5),
            "span_us": round(float(t[:, -1].max()) / 1e3, 2),
            "wg_life_us": round(float(life.mean()) / 1e3, 2),
            "first_stage_us": round(float(first.mean()) / 1e3, 3),
            "kstep_us_mean": round(float(steps.mean()) / 1e3, 3),
            "kstep_us_p90": round(float(np.percentile(steps, 90)) / 1e3, 3),
            "last_step_us": round(float(last.mean()) / 1e3, 3),
            "epilogue_us": round(float(epi.mean()) / 1e3, 3),
            "start_quartiles_us": [round(float(np.percentile(t[:, 0], q)) / 1e3, 2) for q in (25, 50, 75, 100)],
            "mfma_bound_kstep_us": round(1024 / 2.4e3, 3)}), flush=True)
        del A, W, C, tr


if __name__ == "__main__":
    main()
