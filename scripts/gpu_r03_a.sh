#!/bin/bash
# Round-3 checks: train-step parity reports (fp32 + bf16, all geometries), the DP overlap test at
# world 2, the quads-cache and non-finite-gradient tests, the RCCL capture child.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/parity
export IRADS_REPORT_DIR=gpurun_out/parity
run() {  # name, timeout, pytest args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/$name.log | tail -25
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited with $rc"; exit $rc; fi
}
run r03_parity2 900 tests/test_gpu_train_parity.py -m gpu
run r03_new 400 -m gpu tests/test_gpu_drivers.py -k dp_two_ranks tests/test_gpu_swin_fused.py::test_bias_quads_cache_lives_with_its_table tests/test_gpu_dattn_native.py
run r03_rccl 300 -m gpu tests/test_gpu_zz_rccl.py
exit 0
