#!/bin/bash
# wgrad iteration on the GPU box: the split-K weight-gradient tests, the bench line, and a
# kernel trace of a short bench run reduced to per-step wgrad kernel times.
#   scripts/gpu_wgrad_iter.sh <tag>
cd "$(dirname "$0")/.."
tag=${1:-wg}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_swin_fused.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/wgrad_tests_$tag.log 2>&1
rc=$?; tail -3 gpurun_out/wgrad_tests_$tag.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --no-kernels --no-cpu-baseline > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { echo "bench failed"; tail -5 gpurun_out/bench_$tag.err; exit 1; }
tail -1 gpurun_out/bench_$tag.json | cut -c1-260
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_$tag --steps 10 --warmup 3 --no-cpu-baseline --no-kernels || exit 1
python3 scripts/trace_summary.py gpurun_out/prof_$tag/run_kernel_trace.csv.gz --top 200 > gpurun_out/breakdown_$tag.txt
head -1 gpurun_out/breakdown_$tag.txt; grep wgrad gpurun_out/breakdown_$tag.txt
