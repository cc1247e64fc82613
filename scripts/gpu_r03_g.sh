#!/bin/bash
# Table-seeded base-2 forward (4-copy b128 seeds): parity incl. the shifted-row path, timings.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
t() {  # name, pytest args
  local name=$1; shift
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep -E "^FAILED|Error" gpurun_out/$name.log | head -5; tail -1 gpurun_out/$name.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  return 0
}
IRADS_WINATTN_FWD_PC=-1 t g_rt tests/test_gpu_swin.py tests/test_gpu_swin_fused.py tests/test_gpu_train_parity.py
t g_default tests/test_gpu_swin.py -k "window or shifted"
for v in "0 0" "-1 0"; do
  set -- $v
  IRADS_WINATTN_FWD_PC=$1 IRADS_WINATTN_BWD_RC=$2 timeout -k 10 200 python -u scripts/winattn_lab.py > gpurun_out/lab_g_$1_$2.log 2>&1 || exit $?
  echo "fwd=$1 bwd_rc=$2"; grep -v amdgpu.ids gpurun_out/lab_g_$1_$2.log
done
