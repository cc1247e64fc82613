#!/bin/bash
# A/B of two hipBLASLt selection tables on one box: old, new, old, new.
# NEW_TABLE=<csv> (default: ir-ads_amd/irads/tuned/candidate.csv) against the shipped one.
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
for t in old new old new; do
  if [ $t = new ]; then export IRADS_GEMM_TABLE=${NEW_TABLE:-ir-ads_amd/irads/tuned/candidate.csv}; else unset IRADS_GEMM_TABLE; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernels > gpurun_out/ab_$t.log 2>&1 || { echo "bench $t failed"; exit 1; }
  echo "$t $(tail -1 gpurun_out/ab_$t.log | cut -c1-150)"
done
