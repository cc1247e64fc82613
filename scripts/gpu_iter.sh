#!/bin/bash
# Iteration run on the GPU box: given parity files, then a short bench, then a kernel-trace profile.
#   bash scripts/gpu_iter.sh <tag> tests/test_a.py tests/test_b.py ...
cd "$(dirname "$0")/.."
tag=$1; shift
mkdir -p gpurun_out
bash scripts/gpu_tests.sh "$@" || exit $?
for f in "$@"; do grep -q "passed" gpurun_out/$(basename $f .py).log && ! grep -qE "[0-9]+ failed" gpurun_out/$(basename $f .py).log || { echo "parity failures: not benchmarking"; exit 1; }; done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log
PROFILE_TIMEOUT=400 bash scripts/profile_bench.sh prof_$tag --steps 6 --warmup 4 --no-cpu-baseline --profile-only
