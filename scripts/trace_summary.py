"""Summarise a rocprofv3 kernel trace of bench.py.

    python scripts/trace_summary.py gpurun_out/prof3/run_kernel_trace.csv.gz --steps 5 [--match winattn]

Prints the top kernels by time per training step.  Only the last `--steps` steps are
counted: the run is cut at the last `--steps` occurrences of the first AdamW launch.
With --match, it also prints per-launch durations grouped by grid size for the kernels
whose names contain the pattern.
"""
import argparse
import collections
import csv
import gzip


def short(name, n=90):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    name = name.split("(")[0]
    return name if len(name) <= n else name[:n - 3] + "..."


CATS = [("irads::winattn", "winattn (HIP)"), ("irads::dattn", "dattn (HIP)"), ("irads::msda", "msda (HIP)"),
        ("irads::resize", "resize (HIP)"), ("irads::ce_", "cross-entropy (HIP)"), ("irads::", "other HIP"),
        ("Cijk_", "GEMM (hipBLASLt/Tensile)"), ("ck::", "conv (CK)"), ("miopen", "conv (MIOpen)"),
        ("naive_conv", "conv (MIOpen naive)"), ("igemm", "conv (MIOpen igemm)"), ("layer_norm", "layer norm"),
        ("cuComputeGrad", "layer norm"), ("bfloat16_copy", "cast fp32->bf16"), ("bfloat16tofloat32", "cast bf16->fp32"),
        ("adam", "optimizer"), ("reduce_kernel", "reductions"), ("batch_norm", "batch norm"),
        ("Gelu", "gelu"), ("elementwise", "elementwise"), ("rocclr", "runtime copy/fill")]


def category(name):
    low = name.lower()
    for pat, cat in CATS:
        if pat.lower() in low:
            return cat
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--match", default=None)
    ap.add_argument("--categories", action="store_true", help="group kernels into coarse categories")
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    with op(a.trace, "rt") as f:
        rows = [r for r in csv.DictReader(f) if r["Kind"] == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # step boundaries: launches of the fused AdamW kernel (one per step)
    adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"].lower()]
    firsts = [adam[0]] + [b for a_, b in zip(adam, adam[1:]) if b - a_ > 50]
    if len(firsts) > a.steps:
        rows = rows[firsts[-a.steps - 1] + 1:firsts[-1] + 1]
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        tot[r["Kernel_Name"]] += d
        cnt[r["Kernel_Name"]] += 1
    allms = sum(tot.values())
    print(f"kernel time per step: {allms / a.steps:.2f} ms  ({len(rows) / a.steps:.0f} launches/step)")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{v / a.steps:8.3f} ms  {cnt[k] / a.steps:6.1f}x  {short(k)}")
    if a.categories:
        cats = collections.defaultdict(float)
        for k, v in tot.items():
            cats[category(short(k, 400))] += v
        print("-- by category (ms/step)")
        for k, v in sorted(cats.items(), key=lambda kv: -kv[1]):
            print(f"{v / a.steps:8.3f}  {k}")
    if a.match:
        groups = collections.defaultdict(list)
        for r in rows:
            if a.match in r["Kernel_Name"]:
                key = (short(r["Kernel_Name"], 60), r["Grid_Size_X"], r["LDS_Block_Size"], r["VGPR_Count"])
                groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
        for k, v in sorted(groups.items()):
            print(f"{k}: n={len(v)} avg={sum(v) / len(v):.1f} us min={min(v):.1f} max={max(v):.1f}")


if __name__ == "__main__":
    main()
