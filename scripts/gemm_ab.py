"""irads_gemm_nt against hipBLASLt (the shipped TunableOp table) at the Swin-B trunk's C2 shapes:
correctness (relative L2 to the fp32 product; GELU / dGELU epilogues bit for bit against the element
kernels applied to the same GEMM's plain output) and time per call.

    python scripts/gemm_ab.py [--stages 0,1,2,3]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from irads import native as N  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0").split(",") if v]  # besides irads_gemm_nt's
STAGES = ((128, 262144, 2), (256, 65536, 2), (512, 16384, 18), (1024, 4096, 2))


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


def gemm(epi, A, B, bias=None, U=None, C1=None, variant=2):
    M, K = A.shape
    Nn = B.shape[0]
    C0 = torch.empty((M, Nn), device=A.device, dtype=torch.bfloat16)
    N.call("irads_gemm_nt_variant", variant, epi, N.ptr(A), A.stride(0), N.ptr(B), B.stride(0), N.ptr(bias), N.ptr(U),
           0 if U is None else U.stride(0), N.ptr(C0), N.ptr(C1), C0.stride(0), M, Nn, K, N.stream())
    return C0


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def main():
    from irads.gemm_tuning import use_tuned_gemms
    use_tuned_gemms()
    stages = [int(s) for s in (sys.argv[sys.argv.index("--stages") + 1].split(",") if "--stages" in sys.argv
                               else "0,1,2,3".split(","))]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    tot = {"lib": 0.0, "irads": 0.0}
    for si in stages:
        C, M, blocks = STAGES[si]
        for op, K, Nn in (("qkv", C, 3 * C), ("proj", C, C), ("fc1", C, 4 * C), ("fc2", 4 * C, C)):
            A = torch.randn(M, K, device=dev).bfloat16()
            W = (torch.randn(Nn, K, device=dev) * K ** -0.5).bfloat16()
            bias = (torch.randn(Nn, device=dev) * 0.1).bfloat16()
            bias32 = bias.float()
            # forward: y = A Wᵀ + b
            ref32 = torch.addmm(bias32, A.float(), W.float().t())
            lib = F.linear(A, W, bias)
            mine = gemm(0, A, W, bias32)
            row = {"C": C, "op": op, "dir": "fwd", "M": M, "K": K, "N": Nn,
                   "err_lib": rel(lib, ref32), "err_irads": rel(mine, ref32)}
            row["lib_us"] = timed(lambda: F.linear(A, W, bias))
            row["irads_us"] = timed(lambda: gemm(0, A, W, bias32))
            for v in VARIANTS:
                if v >= 4 and Nn % 256:
                    continue
                row[f"irads_v{v}_us"] = timed(lambda: gemm(0, A, W, bias32, variant=v))
                assert torch.equal(gemm(0, A, W, bias32, variant=v), mine)
            if op == "fc1":  # fused GELU epilogue: bit-identical to the element kernel on the same U
                g = torch.empty_like(mine)
                u = gemm(1, A, W, bias32, C1=g)
                assert torch.equal(u, mine), "EPI_GELU's U differs from EPI_BIAS"
                g_ref = torch.empty_like(u)
                N.call("irads_gelu_fwd", N.ptr(u), N.ptr(g_ref), u.numel(), N.stream())
                assert torch.equal(g, g_ref), "EPI_GELU's G differs from irads_gelu_fwd"
                row["irads_gelu_us"] = timed(lambda: gemm(1, A, W, bias32, C1=g))
                row["lib_plus_gelu_us"] = row["lib_us"] + timed(
                    lambda: N.call("irads_gelu_fwd", N.ptr(u), N.ptr(g_ref), u.numel(), N.stream()))
            print(json.dumps({k: (round(v, 6) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
            tot["lib"] += row["lib_us"] * blocks
            tot["irads"] += min(row["irads_us"], row["lib_us"]) * blocks
            # backward: dX = dY W  ->  NT with B = Wᵀ (made once: frozen weights)
            dY = torch.randn(M, Nn, device=dev).bfloat16()
            Wt = W.t().contiguous()
            ref32 = dY.float() @ W.float()
            lib = torch.mm(dY, W)
            mine = gemm(0, dY, Wt)
            row = {"C": C, "op": op, "dir": "bwd", "M": M, "K": Nn, "N": K,
                   "err_lib": rel(lib, ref32), "err_irads": rel(mine, ref32)}
            row["lib_us"] = timed(lambda: torch.mm(dY, W))
            row["irads_us"] = timed(lambda: gemm(0, dY, Wt))
            for v in VARIANTS:
                if v >= 4 and K % 256:
                    continue
                row[f"irads_v{v}_us"] = timed(lambda: gemm(0, dY, Wt, variant=v))
                assert torch.equal(gemm(0, dY, Wt, variant=v), mine)
            if op == "fc2":  # dGELU epilogue (dU of fc1's output U) against irads_gelu_bwd on the same dG
                U = (torch.randn(M, K, device=dev) * 1.5).bfloat16()
                du = gemm(2, dY, Wt, U=U)
                du_ref = torch.empty_like(du)
                N.call("irads_gelu_bwd", N.ptr(U), N.ptr(mine), N.ptr(du_ref), du.numel(), N.stream())
                assert torch.equal(du, du_ref), "EPI_DGELU differs from irads_gelu_bwd"
                row["irads_dgelu_us"] = timed(lambda: gemm(2, dY, Wt, U=U))
                row["lib_plus_gelu_bwd_us"] = row["lib_us"] + timed(
                    lambda: N.call("irads_gelu_bwd", N.ptr(U), N.ptr(mine), N.ptr(du_ref), du.numel(), N.stream()))
            print(json.dumps({k: (round(v, 6) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
            tot["lib"] += row["lib_us"] * blocks
            tot["irads"] += min(row["irads_us"], row["lib_us"]) * blocks
            del A, W, dY, Wt, lib, mine, ref32
            torch.cuda.empty_cache()
    print(json.dumps({"trunk_ms_lib": round(tot["lib"] / 1e3, 3), "trunk_ms_best_of_both": round(tot["irads"] / 1e3, 3)}))


if __name__ == "__main__":
    main()
