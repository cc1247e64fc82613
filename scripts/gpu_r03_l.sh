#!/bin/bash
# MSDA gather backward with the split pass for coarse levels: parity, then the per-kernel trace.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_msda.py tests/test_gpu_dino.py > gpurun_out/l_msda.log 2>&1
rc=$?; echo "msda tests rc=$rc"; grep -E "^FAILED|Error" gpurun_out/l_msda.log | head -5; tail -1 gpurun_out/l_msda.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_msda_iter.sh
