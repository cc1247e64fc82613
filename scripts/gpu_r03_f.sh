#!/bin/bash
# Base-2 scaled window attention (prescaled q, no per-score fma in the forward): parity under the
# table-seeded forward with both backward kernels, kernel timings, then the C2 bench with it.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
t() {  # name, pytest args
  local name=$1; shift
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep -E "^FAILED|Error" gpurun_out/$name.log | head -5; tail -1 gpurun_out/$name.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  return 0
}
IRADS_WINATTN_FWD_PC=-1 t f_rt tests/test_gpu_swin.py tests/test_gpu_swin_fused.py
IRADS_WINATTN_FWD_PC=-1 IRADS_WINATTN_BWD_RC=1 t f_rt_rc tests/test_gpu_swin.py tests/test_gpu_swin_fused.py
for v in "0 0" "-1 0" "-1 1"; do
  set -- $v
  IRADS_WINATTN_FWD_PC=$1 IRADS_WINATTN_BWD_RC=$2 timeout -k 10 200 python -u scripts/winattn_lab.py > gpurun_out/lab_f_$1_$2.log 2>&1 || exit $?
  echo "fwd=$1 bwd_rc=$2"; grep step_avg gpurun_out/lab_f_$1_$2.log
done
IRADS_WINATTN_FWD_PC=-1 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-kernels --no-cpu-baseline > gpurun_out/bench_f.log 2>&1 || { tail -3 gpurun_out/bench_f.log; exit 1; }
tail -1 gpurun_out/bench_f.log | cut -c1-1500
