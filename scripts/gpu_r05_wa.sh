#!/bin/bash
# Round 5: window-attention forward without the row maximum (row-sum guard, libirads_exp.so) against
# the shipped forward (libirads.so), same box, at the C2 step's launch shapes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/winattn_ab.py --variants 0 > gpurun_out/wa_ab_base_r05.log 2>&1 || { echo "base failed"; tail -20 gpurun_out/wa_ab_base_r05.log; exit 1; }
IRADS_LIB=ir-ads_amd/irads/libirads_exp.so timeout -k 10 240 python -u scripts/winattn_ab.py --variants 0 > gpurun_out/wa_ab_exp_r05.log 2>&1 || { echo "exp failed"; tail -20 gpurun_out/wa_ab_exp_r05.log; exit 1; }
timeout -k 10 240 python -u scripts/winattn_ab.py --variants 0 > gpurun_out/wa_ab_base2_r05.log 2>&1 || { echo "base2 failed"; exit 1; }
tail -12 gpurun_out/wa_ab_base_r05.log; echo ---; tail -12 gpurun_out/wa_ab_exp_r05.log; echo ---; tail -12 gpurun_out/wa_ab_base2_r05.log
# the same bench step on both libraries (window-attention periods from the stamps, forward and backward)
IRADS_LIB=ir-ads_amd/irads/libirads_exp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_swin.py tests/test_gpu_winattn_variants.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_wa_exp_r05.log 2>&1 || { echo "exp winattn tests failed"; tail -30 gpurun_out/tests_wa_exp_r05.log; exit 1; }
tail -1 gpurun_out/tests_wa_exp_r05.log
for lib in base exp base2 exp2; do
  L=ir-ads_amd/irads/libirads.so; case $lib in exp*) L=ir-ads_amd/irads/libirads_exp.so;; esac
  IRADS_LIB=$L IRADS_STAMP_DUMP=gpurun_out/stamps_$lib.npz timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-kernels --no-cpu-baseline > gpurun_out/bench_$lib.log 2>&1 || { echo "bench $lib failed"; tail -20 gpurun_out/bench_$lib.log; exit 1; }
  python - "$lib" <<'PY'
import json, sys
r = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], r["value"], r["ms_per_step"], "fwd", r["roofline"]["frac"], r["roofline"]["avg_launch_ms"], "bwd", r["roofline_bwd"]["frac"], r["roofline_bwd"]["avg_launch_ms"])
PY
done
