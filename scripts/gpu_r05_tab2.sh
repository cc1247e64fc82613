#!/bin/bash
# The shipped GEMM table after the 1.05 rule: every entry through its kernel, the C2 step table-vs-off.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_gemm_step.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/tests_tab2_r05.log 2>&1
rc=$?; tail -3 gpurun_out/tests_tab2_r05.log; grep -E "FAILED|ERROR" gpurun_out/tests_tab2_r05.log | head; exit $rc
