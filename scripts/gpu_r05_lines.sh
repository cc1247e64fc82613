#!/bin/bash
# Final-tree bench lines: C2 (no kernel lines, no CPU baseline) and the C3 / C4 workloads.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for w in c2 c3 c4; do
  timeout -k 10 500 python -u bench.py --workload $w --no-kernels --no-cpu-baseline > gpurun_out/bench_line_$w.json 2> gpurun_out/bench_line_$w.err || { echo "bench $w failed"; tail -5 gpurun_out/bench_line_$w.err; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/bench_line_$w.json').read().strip().splitlines()[-1]); print('$w', r['value'], r['ms_per_step'], r['config'].get('workload'))"
done
