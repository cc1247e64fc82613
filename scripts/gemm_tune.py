"""Build irads.gemm's selection table: irads_gemm_nt against hipBLASLt (the shipped TunableOp table)
on every trunk projection shape of BASELINE.json's C2 (Swin-B, 8 x 512², rgb + dte batched), C4
(Swin-L, 4 x 480x640) and C3 (Swin-B, 4 x 512²) steps, forward y = x Wᵀ + b and backward dX = dY W, in interleaved rounds in
one process (median of 5 rounds x 10 calls each).  A shape goes to irads_gemm_nt when its median is
≥ 5 % below hipBLASLt's and its error against the fp32 product is no worse than 1.5x hipBLASLt's.
The FFN's fused pairs (fc1 + GELU epilogue, fc2 dX + GELU' epilogue) are timed against the better
unfused arm (hipBLASLt or irads_gemm_nt, then the element pass) and kept on the same 5 % margin.
Each irads arm tries the tilings in VARIANTS and the table keeps the winner's: [dir, M, N, K, variant].

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
         [("c4", 192 * 2 ** s, 153600 // 4 ** s) for s in range(4)] + \
         [("c3", 128 * 2 ** s, 131072 // 4 ** s) for s in range(4)]  # C3: Swin-B 512², 4 per GPU


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


# irads_gemm_nt wins a shape when its median is within WIN[cfg] of the library arm's.  In the C2 step
# it runs faster than in this isolated timing, and the 1.05 bound measured 0.1 ms per C2 step better
# than 0.95 (profiles/r05_bench_le105_*.json); for the C3 / C4 shapes the same bound measured 0.18 /
# 0.07 ms per step slower (profiles/r05_bench_ab_c3_*.json, _c4_*), so they keep 0.95.
WIN = {"c2": 1.05, "c3": 0.95, "c4": 0.95}
# irads_gemm_nt_variant tilings tried per shape (4 only where N % 256 == 0); IRADS_TUNE_VARIANTS=0,1,2,3,4
VARIANTS = tuple(int(v) for v in os.environ.get("IRADS_TUNE_VARIANTS", "2,4").split(","))


def nt(A, B, bias32, v=2):
    M, K = A.shape
    out = torch.empty((M, B.shape[0]), device=A.device, dtype=torch.bfloat16)
    N.call("irads_gemm_nt_variant", v, 0, N.ptr(A), A.stride(0), N.ptr(B), B.stride(0), N.ptr(bias32), None, 0,
           N.ptr(out), None, out.stride(0), M, B.shape[0], K, N.stream())
    return out


def gelu(u):
    g = torch.empty_like(u)
    N.call("irads_gelu_fwd", N.ptr(u), N.ptr(g), u.numel(), N.stream())
    return g


def gelu_bwd(u, dg):
    du = torch.empty_like(dg)
    N.call("irads_gelu_bwd", N.ptr(u), N.ptr(dg), N.ptr(du), du.numel(), N.stream())
    return du


def fused_rows(cfg, M, C, C4, A, W1, b16, b32):
    """The FFN's fused pairs against the better unfused arm: fc1 + GELU (U, G), and fc2's dX + GELU'
    (dU; fc2 = W2 (C, 4C), so its dX is (M, 4C) = dF (M, C) · W2 with U of fc1's output shape)."""
    out, keys = [], []
    vs = [v for v in VARIANTS if G.kernel_fits(C4, C, v)]
    lib_fc1 = lambda: gelu(F.linear(A, W1, b16))  # noqa: E731
    ir_fc1 = lambda: gelu(nt(A, W1, b32))  # noqa: E731

    def fused_fc1(v):
        u = torch.empty((M, C4), device=A.device, dtype=torch.bfloat16)
        g = torch.empty_like(u)
        N.call("irads_gemm_nt_variant", v, 1, N.ptr(A), A.stride(0), N.ptr(W1), W1.stride(0), N.ptr(b32), None, 0,
               N.ptr(u), N.ptr(g), u.stride(0), M, C4, C, N.stream())
        return g
    W2 = (torch.randn(C, C4, device=A.device) * C4 ** -0.5).bfloat16()  # fc2's weight (C, 4C)
    W2t = W2.t().contiguous()  # (4C, C)
    dF = torch.randn(M, C, device=A.device).bfloat16()
    U = (torch.randn(M, C4, device=A.device) * 1.5).bfloat16()
    lib_fc2 = lambda: gelu_bwd(U, torch.mm(dF, W2))  # noqa: E731
    ir_fc2 = lambda: gelu_bwd(U, nt(dF, W2t, None))  # noqa: E731

    def fused_fc2(v):
        du = torch.empty((M, C4), device=A.device, dtype=torch.bfloat16)
        N.call("irads_gemm_nt_variant", v, 2, N.ptr(dF), dF.stride(0), N.ptr(W2t), W2t.stride(0), None, N.ptr(U),
               U.stride(0), N.ptr(du), None, du.stride(0), M, C4, C, N.stream())
        return du
    for d, key, lib_arm, ir_arm, fused in (("fwd_gelu", ("fwd_gelu", M, C4, C), lib_fc1, ir_fc1, fused_fc1),
                                           ("bwd_dgelu", ("bwd_dgelu", M, C4, C), lib_fc2, ir_fc2, fused_fc2)):
        if not vs:
            continue
        arms = [lib_arm, ir_arm] + [lambda v=v: fused(v) for v in vs]
        ref = arms[0]()
        e = [rel(a(), ref) for a in arms]
        for a in arms:
            a(), a()
        ts = [[] for _ in arms]
        for _ in range(5):
            for j, a in enumerate(arms):
                ts[j].append(timed(a))
        med = [statistics.median(t) for t in ts]
        jb = 2 + min(range(len(vs)), key=lambda j: med[2 + j])
        win = med[jb] <= WIN[cfg] * min(med[0], med[1]) and e[jb] <= 2e-2
        row = {"cfg": cfg, "op": "fc1+gelu" if d == "fwd_gelu" else "fc2+dgelu", "dir": d, "M": M, "N": C4, "K": C,
               "lib_plus_pass_us": round(med[0], 2), "irads_plus_pass_us": round(med[1], 2),
               **{f"fused_v{v}_us": round(med[2 + j], 2) for j, v in enumerate(vs)},
               "variant": vs[jb - 2], "fused_vs_lib_rel": round(e[jb], 6), "irads": win}
        print(json.dumps(row), flush=True)
        out.append(row)
        if win:
            keys.append(list(key) + [vs[jb - 2]])
    return out, keys


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
                    ("fwd", ("fwd", M, Nn, K), lambda: F.linear(A, W, b16), lambda v: nt(A, W, b32, v),
                     lambda: torch.addmm(b32, A.float(), W.float().t())),
                    ("bwd", ("bwd", M, K, Nn), lambda: torch.mm(dY, W), lambda v: nt(dY, Wt, None, v),
                     lambda: dY.float() @ W.float())):
                if key in seen or not G.kernel_fits(key[2], key[3]):
                    continue
                seen.add(key)
                vs = [v for v in VARIANTS if G.kernel_fits(key[2], key[3], v)]
                arms = [lib] + [lambda v=v, mine=mine: mine(v) for v in vs]
                r32 = ref()
                e = [rel(a(), r32) for a in arms]
                del r32
                for _ in range(2):
                    for a in arms:
                        a()
                ts = [[] for _ in arms]
                for _ in range(5):
                    for j, a in enumerate(arms):
                        ts[j].append(timed(a))
                med = [statistics.median(t) for t in ts]
                jb = 1 + min(range(len(vs)), key=lambda j: med[1 + j])
                win = med[jb] <= WIN[cfg] * med[0] and e[jb] <= 1.5 * e[0] + 1e-4
                row = {"cfg": cfg, "op": op, "dir": d, "M": key[1], "N": key[2], "K": key[3], "lib_us": round(med[0], 2),
                       **{f"irads_v{v}_us": round(med[1 + j], 2) for j, v in enumerate(vs)}, "variant": vs[jb - 1],
                       "err_lib": round(e[0], 6), "err_irads": round(e[jb], 6), "irads": win}
                print(json.dumps(row), flush=True)
                rows.append(row)
                if win:
                    keys.append(list(key) + [vs[jb - 1]])
            if op == "fc1" and G.kernel_fits(Nn, K):
                rows_, keys_ = fused_rows(cfg, M, K, Nn, A, W, b16, b32)
                rows += rows_
                keys += keys_
            del A, W, Wt, dY
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    with open(out_path, "w") as fh:
        json.dump({"device": torch.cuda.get_device_name(0), "rule": f"median irads <= WIN[cfg] x median hipBLASLt, WIN = {WIN}",
                   "irads": keys, "measured": rows}, fh, indent=1)
    print(json.dumps({"irads_shapes": len(keys), "of": len(rows)}))


if __name__ == "__main__":
    main()
