#!/bin/bash
# Cross-entropy kernels on v_exp_f32: the seghead / loss parity tests, then the bench line and a kernel trace.
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v -rfs --timeout 240 --timeout-method thread -m gpu tests/test_gpu_seghead.py tests/test_gpu_train_parity.py > gpurun_out/r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r_tests.log | head -8; tail -1 gpurun_out/r_tests.log
[ $rc -ne 0 ] && exit $rc
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_r03r --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
f=$(find gpurun_out/prof_r03r -name "*kernel_trace.csv.gz" | head -1); python3 scripts/trace_summary.py "$f" --steps 4 --top 200 > gpurun_out/step_breakdown_r03r.txt 2>&1; head -1 gpurun_out/step_breakdown_r03r.txt; grep -E "ce_|resize" gpurun_out/step_breakdown_r03r.txt | head
