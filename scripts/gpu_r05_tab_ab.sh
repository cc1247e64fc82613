#!/bin/bash
# In-step A/B of the GELU table: the default bench step with IRADS_GEMM_GELU_TABLE=0 and without, twice.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for mode in formula table formula2 table2; do
  env=""; case $mode in formula*) export IRADS_GEMM_GELU_TABLE=0;; *) unset IRADS_GEMM_GELU_TABLE;; esac
  timeout -k 10 400 python -u bench.py --no-kernels --no-cpu-baseline --steps 50 > gpurun_out/bench_tab_$mode.json 2> gpurun_out/bench_tab_$mode.err || { echo "bench $mode failed"; tail -5 gpurun_out/bench_tab_$mode.err; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/bench_tab_$mode.json').read().strip().splitlines()[-1]); print('$mode', r['value'], r['ms_per_step'])"
done
