#!/bin/bash
# Round 5 combined batch: GEMM variant 5 (tests + A/B), then scripts/gpu_r05_b.sh (window-attention
# A/B and benches on both libraries, forward traffic PMC, MSDA trace + PMC).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_gemm_r05.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/tests_gemm_r05.log; exit 1; }
tail -1 gpurun_out/tests_gemm_r05.log
GEMM_VARIANTS=4,5 timeout -k 10 300 python -u scripts/gemm_ab.py --stages 0,1,2,3 > gpurun_out/gemm_ab_r05b.log 2>&1 || { echo "gemm_ab failed rc=$?"; tail -30 gpurun_out/gemm_ab_r05b.log; exit 1; }
echo gemm_ab ok
bash scripts/gpu_r05_b.sh
