#!/bin/bash
# C3 and C4 throughput lines on the final tree (builder-run; the driver measures C2).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for wl in c3 c4; do
  timeout -k 10 500 python -u bench.py --workload $wl --no-kernels > gpurun_out/bench_r05_$wl.json 2> gpurun_out/bench_r05_$wl.err || { echo "$wl failed"; tail -5 gpurun_out/bench_r05_$wl.err; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/bench_r05_$wl.json').read().strip().splitlines()[-1]); print('$wl', r['value'], r['ms_per_step'], r.get('roofline', {}).get('frac'))"
done
