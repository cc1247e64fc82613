#!/bin/bash
# Re-tune the step's GEMM selection (TunableOp, longer per-shape timing) and A/B the bench line:
# shipped table / hipBLASLt heuristic / new table, interleaved on one box.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/tune_gemms.py --out gpurun_out/tunableop_new.csv --max-ms ${1:-100} > gpurun_out/tune_new.log 2>&1 || { tail gpurun_out/tune_new.log; exit 1; }
tail -2 gpurun_out/tune_new.log
ls -la gpurun_out/tunableop_new.csv* 2>/dev/null
new=$(ls gpurun_out/tunableop_new*.csv | head -1)
for rep in 1 2; do
  for arm in shipped heuristic new; do
    case $arm in
      shipped) env="";;
      heuristic) env="";;
      new) env="IRADS_GEMM_TABLE=$new";;
    esac
    extra=""; [ $arm = heuristic ] && extra="--no-tuned-gemms"
    env $env timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-kernels --no-cpu-baseline $extra > gpurun_out/bench_gemm_${arm}_$rep.log 2>&1 || { echo "bench $arm failed"; tail -3 gpurun_out/bench_gemm_${arm}_$rep.log; exit 1; }
    echo "$arm $rep $(tail -1 gpurun_out/bench_gemm_${arm}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
