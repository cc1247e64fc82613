#!/bin/bash
# BN finalize / DropPath kernels: their GPU tests, then the default bench step with the previous
# host code (abtmp_old: HEAD's python, the same libirads.so) and the new, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_seghead.py tests/test_gpu_swin_fused.py > gpurun_out/tests_glue.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/tests_glue.log | head -20; tail -5 gpurun_out/tests_glue.log; exit 1; }
tail -1 gpurun_out/tests_glue.log
LIB=$PWD/ir-ads_amd/irads/libirads.so
for mode in old new old2 new2; do
  case $mode in old*) B=abtmp_old/bench.py;; *) B=bench.py;; esac
  IRADS_LIB=$LIB timeout -k 10 400 python -u $B --no-kernels --no-cpu-baseline --steps 50 > gpurun_out/bench_glue_$mode.json 2> gpurun_out/bench_glue_$mode.err || { echo "bench $mode failed"; tail -5 gpurun_out/bench_glue_$mode.err; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/bench_glue_$mode.json').read().strip().splitlines()[-1]); print('$mode', r['value'], r['ms_per_step'])"
done
