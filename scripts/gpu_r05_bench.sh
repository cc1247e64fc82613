#!/bin/bash
# Round 5: the default bench line (C2 step + kernel lines incl. the C5 detector step + cpu_baseline).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r05_full.json 2> gpurun_out/bench_r05_full.err
rc=$?
tail -5 gpurun_out/bench_r05_full.err
echo "bench rc=$rc"
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/bench_r05_full.json").read().strip().splitlines()[-1])
print(r["value"], r["ms_per_step"], "fwd", r["roofline"]["frac"], "bwd", r["roofline_bwd"]["frac"], "gemm", r.get("roofline_gemm", {}).get("frac"))
for k, v in r.get("kernels", {}).items():
    print(k, {kk: v.get(kk) for kk in ("frac", "avg_launch_ms", "ms_per_step", "images_per_s", "error")} if isinstance(v, dict) else v)
print(r.get("cpu_baseline"))
PY
