#!/bin/bash
# Bench + evidence on one box: default bench line, kernel-trace stats of a short run, and the
# window-attention PMC passes (HBM bytes + wave states).  Usage: scripts/gpu_bench_round.sh <tag>
cd "$(dirname "$0")/.."
tag=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { echo "bench failed"; tail -5 gpurun_out/bench_$tag.err; exit 1; }
tail -1 gpurun_out/bench_$tag.json | cut -c1-600
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_$tag --steps 10 --warmup 3 --no-cpu-baseline --no-kernels || exit 1
bash scripts/pmc_winattn.sh > gpurun_out/pmc_$tag.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_$tag.log; exit 1; }
tail -25 gpurun_out/pmc_$tag.log
