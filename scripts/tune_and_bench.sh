#!/bin/bash
# A/B of the shipped hipBLASLt selection table (RETUNE=1 regenerates it first).
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
if [ -n "$RETUNE" ]; then
  timeout -k 10 900 python scripts/tune_gemms.py --out gpurun_out/tunableop_mi355x0.csv --steps 2 --max-ms 30 > gpurun_out/tune.log 2>&1 || { echo tune failed; tail -20 gpurun_out/tune.log; exit 1; }
  tail -3 gpurun_out/tune.log
  cp gpurun_out/tunableop_mi355x0.csv ir-ads_amd/irads/tuned/
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_tuned.log 2>&1 || { echo bench failed; tail gpurun_out/bench_tuned.log; exit 1; }
tail -1 gpurun_out/bench_tuned.log | cut -c1-400
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tuned-gemms > gpurun_out/bench_untuned.log 2>&1 || { echo bench2 failed; tail gpurun_out/bench_untuned.log; exit 1; }
tail -1 gpurun_out/bench_untuned.log | cut -c1-400
