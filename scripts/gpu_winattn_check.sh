#!/bin/bash
# window-attention kernel iteration: parity suites touching it, then per-stage timing (new vs chunked)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_swin_fused.py tests/test_gpu_swin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/winattn_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/winattn_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/kbench.py --only winattn > gpurun_out/kbench_winattn_new.log 2>&1 || exit $?
IRADS_WINATTN_CHUNKED=1 timeout -k 10 200 python -u scripts/kbench.py --only winattn > gpurun_out/kbench_winattn_old.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k c2 > gpurun_out/train_parity.log 2>&1
echo "parity rc=$?"; tail -2 gpurun_out/train_parity.log
