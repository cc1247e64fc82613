#!/bin/bash
# Split-K weight gradients: the target workgroup count (IRADS_WGRAD_WGS) in the C2 step, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for mode in 1024 512 256 1024b 512b 256b; do
  export IRADS_WGRAD_WGS=${mode%b}
  timeout -k 10 400 python -u bench.py --no-kernels --no-cpu-baseline --steps 50 > gpurun_out/bench_wg_$mode.json 2> gpurun_out/bench_wg_$mode.err || { echo "bench $mode failed"; tail -5 gpurun_out/bench_wg_$mode.err; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/bench_wg_$mode.json').read().strip().splitlines()[-1]); print('$mode', r['value'], r['ms_per_step'])"
done
