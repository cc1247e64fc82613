#!/bin/bash
# Fused FFN GEMM + GELU kernels: tests, then the A/B lab.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ffn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ffn_test_$1.log 2>&1; rc=$?
tail -15 gpurun_out/ffn_test_$1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ffn_ab.py > gpurun_out/ffn_ab_$1.log 2>&1 || { echo lab failed; tail -20 gpurun_out/ffn_ab_$1.log; exit 1; }
cat gpurun_out/ffn_ab_$1.log
