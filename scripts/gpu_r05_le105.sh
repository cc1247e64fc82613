#!/bin/bash
# Re-tune the GEMM table over all five tilings, then the default bench step with the shipped table and
# with the new one, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
true
true
for mode in ship new ship2 new2; do
  case $mode in new*) export IRADS_GEMM_SELECT=$PWD/ir-ads_amd/irads/tuned/irads_gemm_select_le105.json;; *) unset IRADS_GEMM_SELECT;; esac
  timeout -k 10 400 python -u bench.py --no-kernels --no-cpu-baseline --steps 50 > gpurun_out/bench_le105_$mode.json 2> gpurun_out/bench_le105_$mode.err || { echo "bench $mode failed"; tail -5 gpurun_out/bench_le105_$mode.err; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/bench_le105_$mode.json').read().strip().splitlines()[-1]); print('$mode', r['value'], r['ms_per_step'])"
done
