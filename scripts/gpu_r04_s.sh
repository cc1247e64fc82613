#!/bin/bash
# Re-tune the TunableOp table on the current step (its GEMM set changed: trunk shapes on irads_gemm_nt,
# the head's fp32 composition products) and A/B the bench line: shipped table vs the new one.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/tune_gemms.py --out gpurun_out/tunableop_new.csv --max-ms ${1:-100} > gpurun_out/tune_new.log 2>&1 || { tail gpurun_out/tune_new.log; exit 1; }
tail -2 gpurun_out/tune_new.log
new=$(ls gpurun_out/tunableop_new*.csv | head -1)
for rep in 1 2; do
  for arm in shipped new; do
    env=""; [ $arm = new ] && env="IRADS_GEMM_TABLE=$new"
    env $env timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-kernels --no-cpu-baseline > gpurun_out/bench_tt_${arm}_$rep.log 2>&1 || { echo "bench $arm failed"; tail -3 gpurun_out/bench_tt_${arm}_$rep.log; exit 1; }
    echo "$arm $rep $(tail -1 gpurun_out/bench_tt_${arm}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
