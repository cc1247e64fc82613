#!/bin/bash
# GELU / GELU' by table in the 256 x 256 GEMM epilogues: bit-exactness, then table vs formula timing.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_gemm_tab.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/tests_gemm_tab.log; exit 1; }
tail -1 gpurun_out/tests_gemm_tab.log
for i in 1 2; do
  IRADS_GEMM_GELU_TABLE=0 timeout -k 10 120 python -u scripts/gelu_table_ab.py > gpurun_out/gelutab_formula_$i.log 2>&1 || exit 1
  timeout -k 10 120 python -u scripts/gelu_table_ab.py > gpurun_out/gelutab_table_$i.log 2>&1 || exit 1
  grep mode gpurun_out/gelutab_formula_$i.log gpurun_out/gelutab_table_$i.log | cut -d: -f2-
done
