#!/bin/bash
# Round-3 parity checks: training-step parity (reports under gpurun_out/parity), DAttn AMP path
# incl. Swin-L stage geometries, MSF evaluation parity, the C1 evaluation driver.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/parity
export IRADS_REPORT_DIR=gpurun_out/parity
run() {  # name, timeout, pytest args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest -v -s --timeout 300 --timeout-method thread "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^msf|^dp " gpurun_out/$name.log | tail -30
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited with $rc"; exit $rc; fi
}
run r03_parity4 900 -m gpu tests/test_gpu_train_parity.py
run r03_amp 400 -m gpu tests/test_gpu_dattn_native.py -k amp_path
run r03_msf 600 -m gpu tests/test_gpu_drivers.py -k "msf or c1"
exit 0
