"""Per-kernel, per-grid mean durations from a rocprofv3 kernel trace (csv or csv.gz).

    python scripts/kernel_grid_stats.py <trace> <regex> [--steps N]
"""
import collections
import csv
import gzip
import re
import sys


def main():
    path, pat = sys.argv[1], re.compile(sys.argv[2])
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 1
    op = gzip.open if path.endswith(".gz") else open
    d = collections.defaultdict(list)
    with op(path, "rt") as fh:
        rows = [r for r in csv.DictReader(fh) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last `steps` training steps only (bench traces: cut at the fused AdamW launch, one per step)
    adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"].lower()]
    if adam:
        firsts = [adam[0]] + [b for a_, b in zip(adam, adam[1:]) if b - a_ > 50]
        if len(firsts) > steps:
            rows = rows[firsts[-steps - 1] + 1:firsts[-1] + 1]
    if True:
        for r in rows:
            n = r["Kernel_Name"]
            if not pat.search(n):
                continue
            name = re.sub(r"\(.*$", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))
            key = (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"])
            d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(d.items()):
        print(f"{k[0]:60s} grid {k[1]:>8s} x {k[2]:>4s} wg {k[3]:>5s}: n={len(v):4d} avg {sum(v) / len(v):8.1f} us"
              f"  per step {sum(v) / steps:9.1f} us")


if __name__ == "__main__":
    main()
