"""Build irads.gemm's selection table: irads_gemm_nt against hipBLASLt (the shipped TunableOp table)
on every trunk projection shape of BASELINE.json's C2 (Swin-B, 8 x 512², rgb + dte batched) and C4
(Swin-L, 4 x 480x640) steps, forward y = x Wᵀ + b and backward dX = dY W, in interleaved rounds in
one process (median of 5 rounds x 10 calls each).  A shape goes to irads_gemm_nt when its median is
≥ 5 % below hipBLASLt's and its error against the fp32 product is no worse than 1.5x hipBLASLt's.

    python scripts/gemm_tune.py [out.json]    (default gpurun_out/irads_gemm_select_mi355x.json;
                                               copy it to ir-ads_amd/irads/tuned/ to ship it)
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from irads import gemm as G  # noqa: E402
from irads import native as N  # noqa: E402

# (config, C, tokens of the batched rgb + dte stage input)
STAGES = [("c2", 128 * 2 ** s, 262144 // 4 ** s) for s in range(4)] + \
         [("c4", 192 * 2 ** s, 153600 // 4 ** s) for s in range(4)]


def timed(fn, reps=10):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def nt(A, B, bias32):
    M, K = A.shape
    out = torch.empty((M, B.shape[0]), device=A.device, dtype=torch.bfloat16)
    N.call("irads_gemm_nt", 0, N.ptr(A), A.stride(0), N.ptr(B), B.stride(0), N.ptr(bias32), None, 0, N.ptr(out),
           None, out.stride(0), M, B.shape[0], K, N.stream())
    return out


def main():
    from irads.gemm_tuning import use_tuned_gemms
    use_tuned_gemms()
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join("gpurun_out", "irads_gemm_select_mi355x.json")
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    keys, rows, seen = [], [], set()
    for cfg, C, M in STAGES:
        for op, K, Nn in (("qkv", C, 3 * C), ("proj", C, C), ("fc1", C, 4 * C), ("fc2", 4 * C, C)):
            A = torch.randn(M, K, device=dev).bfloat16()
            W = (torch.randn(Nn, K, device=dev) * K ** -0.5).bfloat16()
            b16 = (torch.randn(Nn, device=dev) * 0.1).bfloat16()
            b32 = b16.float()
            Wt = W.t().contiguous()
            dY = torch.randn(M, Nn, device=dev).bfloat16()
            for d, key, lib, mine, ref in (
                    ("fwd", ("fwd", M, Nn, K), lambda: F.linear(A, W, b16), lambda: nt(A, W, b32),
                     lambda: torch.addmm(b32, A.float(), W.float().t())),
                    ("bwd", ("bwd", M, K, Nn), lambda: torch.mm(dY, W), lambda: nt(dY, Wt, None),
                     lambda: dY.float() @ W.float())):
                if key in seen or not G.kernel_fits(key[2], key[3]):
                    continue
                seen.add(key)
                r32 = ref()
                e_lib, e_ir = rel(lib(), r32), rel(mine(), r32)
                del r32
                for _ in range(2):
                    lib(), mine()
                t_lib, t_ir = [], []
                for _ in range(5):
                    t_lib.append(timed(lib))
                    t_ir.append(timed(mine))
                ml, mi = statistics.median(t_lib), statistics.median(t_ir)
                win = mi < 0.95 * ml and e_ir <= 1.5 * e_lib + 1e-4
                row = {"cfg": cfg, "op": op, "dir": d, "M": key[1], "N": key[2], "K": key[3], "lib_us": round(ml, 2),
                       "irads_us": round(mi, 2), "err_lib": round(e_lib, 6), "err_irads": round(e_ir, 6),
                       "irads": win}
                print(json.dumps(row), flush=True)
                rows.append(row)
                if win:
                    keys.append(list(key))
            del A, W, Wt, dY
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    with open(out_path, "w") as fh:
        json.dump({"device": torch.cuda.get_device_name(0), "rule": "median irads < 0.95 median hipBLASLt",
                   "irads": keys, "measured": rows}, fh, indent=1)
    print(json.dumps({"irads_shapes": len(keys), "of": len(rows)}))


if __name__ == "__main__":
    main()
