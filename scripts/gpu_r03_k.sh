#!/bin/bash
# stride-20 bias quads in both window-attention directions; MSDA gather with records one chunk ahead.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
t() {  # name, pytest args
  local name=$1; shift
  timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu "$@" > gpurun_out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep -E "^FAILED|Error" gpurun_out/$name.log | head -5; tail -1 gpurun_out/$name.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  return 0
}
t k_swin tests/test_gpu_swin.py tests/test_gpu_swin_fused.py tests/test_gpu_msda.py tests/test_gpu_dino.py
timeout -k 10 200 python -u scripts/winattn_lab.py > gpurun_out/lab_k.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/lab_k.log
bash scripts/gpu_msda_iter.sh || exit $?
IRADS_PMC_KIND=fwd bash scripts/pmc_winattn_kind.sh r03k || exit $?
