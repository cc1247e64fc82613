#!/bin/bash
# window-attention kernel iteration: the parity suites touching it, then graph-timed per-stage kernels
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=${1:-wa}
timeout -k 10 400 python -u -m pytest tests/test_gpu_swin_fused.py tests/test_gpu_swin.py tests/test_gpu_train_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/winattn_tests_$tag.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/winattn_tests_$tag.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/winattn_lab.py > gpurun_out/winattn_lab_$tag.log 2>&1 || exit $?
cat gpurun_out/winattn_lab_$tag.log | grep -v amdgpu.ids
