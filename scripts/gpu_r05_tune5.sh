#!/bin/bash
# Re-tune the GEMM table over all five tilings, then the default bench step with the shipped table and
# with the new one, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
IRADS_TUNE_VARIANTS=0,1,2,3,4 timeout -k 10 900 python -u scripts/gemm_tune.py gpurun_out/irads_gemm_select_all5.json > gpurun_out/gemm_tune5.log 2>&1 || { echo tune failed; tail -5 gpurun_out/gemm_tune5.log; exit 1; }
tail -1 gpurun_out/gemm_tune5.log
for mode in ship new ship2 new2; do
  case $mode in new*) export IRADS_GEMM_SELECT=$PWD/gpurun_out/irads_gemm_select_all5.json;; *) unset IRADS_GEMM_SELECT;; esac
  timeout -k 10 400 python -u bench.py --no-kernels --no-cpu-baseline --steps 50 > gpurun_out/bench_t5_$mode.json 2> gpurun_out/bench_t5_$mode.err || { echo "bench $mode failed"; tail -5 gpurun_out/bench_t5_$mode.err; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/bench_t5_$mode.json').read().strip().splitlines()[-1]); print('$mode', r['value'], r['ms_per_step'])"
done
