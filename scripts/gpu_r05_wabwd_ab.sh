#!/bin/bash
# Window-attention backward: persistent workgroup target (IRADS_WINATTN_BWD_WGS) in the C2 step, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for mode in 256 384 512 256b 384b 512b; do
  export IRADS_WINATTN_BWD_WGS=${mode%b}
  timeout -k 10 400 python -u bench.py --no-kernels --no-cpu-baseline --steps 50 > gpurun_out/bench_wab_$mode.json 2> gpurun_out/bench_wab_$mode.err || { echo "bench $mode failed"; tail -5 gpurun_out/bench_wab_$mode.err; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/bench_wab_$mode.json').read().strip().splitlines()[-1]); print('$mode', r['value'], r['ms_per_step'])"
done
