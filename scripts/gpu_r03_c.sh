#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/parity
export IRADS_REPORT_DIR=gpurun_out/parity
run() {  # name, timeout, pytest args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest -v -s --timeout 300 --timeout-method thread "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " gpurun_out/$name.log | cut -c1-600 | tail -30
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited with $rc"; exit $rc; fi
}
run r03_parity5 900 -m gpu tests/test_gpu_train_parity.py
run r03_keys2 400 -m gpu tests/test_gpu_swin.py::test_dattn_fp32_more_than_1024_keys tests/test_gpu_dattn_native.py::test_dattn_attention_core_many_keys_vs_fp64
exit 0
