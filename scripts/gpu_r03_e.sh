#!/bin/bash
# Window-attention variants (table-seeded forward, persistent forward, per-item backward) and the
# MSDA head-per-XCD mapping: parity tests under each, then kernel timings.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
t() {  # name, pytest args
  local name=$1; shift
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/$name.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  return 0
}
IRADS_WINATTN_FWD_PC=-1 IRADS_WINATTN_BWD_RC=1 t e_new tests/test_gpu_swin.py tests/test_gpu_swin_fused.py
t e_msda tests/test_gpu_msda.py tests/test_gpu_dino.py
for v in "0 0" "-1 1" "4 1"; do
  set -- $v
  IRADS_WINATTN_FWD_PC=$1 IRADS_WINATTN_BWD_RC=$2 timeout -k 10 200 python -u scripts/winattn_lab.py > gpurun_out/lab_$1_$2.log 2>&1 || exit $?
  echo "fwd=$1 bwd_rc=$2"; grep -v amdgpu.ids gpurun_out/lab_$1_$2.log
done
timeout -k 10 200 python -u scripts/msda_bench.py > gpurun_out/msda_bench_e.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/msda_bench_e.log | cut -c1-250
