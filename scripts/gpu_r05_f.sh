#!/bin/bash
# Round 5: bench with stamped periods vs the kernel trace of the same tree.
cd "$(dirname "$0")/.."
tag=${1:-r05f}
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -q -rfs --timeout 240 --timeout-method thread -k "gelu or dispatch" > gpurun_out/tests_${tag}.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 gpurun_out/tests_${tag}.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 500 python bench.py --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { echo bench failed; tail gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log | cut -c1-200
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_$tag --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv.gz" | head -1); python3 scripts/trace_summary.py "$f" --steps 4 --match winattn > gpurun_out/step_breakdown_$tag.txt 2>&1; head -1 gpurun_out/step_breakdown_$tag.txt
