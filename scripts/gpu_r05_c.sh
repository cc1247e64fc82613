#!/bin/bash
# Round 5: DAttn pass-Q 64-bit table gradient + stamps without entry stores; parity; bench; trace.
cd "$(dirname "$0")/.."
tag=${1:-r05c}
mkdir -p gpurun_out/parity_$tag
export IRADS_REPORT_DIR=gpurun_out/parity_$tag
timeout -k 10 900 python -u -m pytest tests/test_gpu_dattn_native.py tests/test_gpu_determinism.py tests/test_gpu_train_parity.py \
    -m gpu -v -rfs --timeout 400 --timeout-method thread -s > gpurun_out/tests_${tag}.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/tests_${tag}.log | head; tail -2 gpurun_out/tests_${tag}.log
grep -E "^rpe |^q |^k " gpurun_out/tests_${tag}.log | head -12
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 500 python bench.py --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { echo bench failed; tail gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log | cut -c1-300
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_$tag --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv.gz" | head -1); python3 scripts/trace_summary.py "$f" --steps 4 --match "winattn|dattn_attn" > gpurun_out/step_breakdown_$tag.txt 2>&1; head -3 gpurun_out/step_breakdown_$tag.txt
