#!/bin/bash
# C3 / C4 steps: the current GEMM table against the previous (5 %-faster rule) one, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for wl in c3 c4; do
for mode in new old new2 old2; do
  case $mode in old*) export IRADS_GEMM_SELECT=$PWD/ir-ads_amd/irads/tuned/irads_gemm_select_old.json;; *) unset IRADS_GEMM_SELECT;; esac
  timeout -k 10 400 python -u bench.py --workload $wl --no-kernels --no-cpu-baseline --steps 50 > gpurun_out/bench_ab_${wl}_$mode.json 2> gpurun_out/bench_ab_${wl}_$mode.err || { echo "$wl $mode failed"; tail -5 gpurun_out/bench_ab_${wl}_$mode.err; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/bench_ab_${wl}_$mode.json').read().strip().splitlines()[-1]); print('$wl $mode', r['value'], r['ms_per_step'])"
done
done
