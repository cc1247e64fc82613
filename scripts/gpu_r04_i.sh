#!/bin/bash
# MSDA non-temporal streaming A/B: the MSDA tests with IRADS_MSDA_NT=1, then the bench's MSDA kernel
# lines with NT off / on / off (interleaved, to see the box's drift).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
IRADS_MSDA_NT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_msda.py -x -q --timeout 240 --timeout-method thread > gpurun_out/msda_nt_tests_$1.log 2>&1; rc=$?
tail -2 gpurun_out/msda_nt_tests_$1.log
[ $rc -ne 0 ] && exit $rc
for nt in 0 1 0 1; do
  IRADS_MSDA_NT=$nt timeout -k 10 200 python -u scripts/msda_bench.py > gpurun_out/msda_nt${nt}_$1.log 2>&1 || { tail gpurun_out/msda_nt${nt}_$1.log; exit 1; }
  echo "NT=$nt"; grep -o '^[a-z_]* {"bound": "hbm", "achieved": [0-9.]*, "peak": 8000.0, "unit": "GB/s", "frac": [0-9.]*, "avg_launch_ms": [0-9.]*' gpurun_out/msda_nt${nt}_$1.log | sed 's/"bound": "hbm", //; s/"peak": 8000.0, "unit": "GB\/s", //'
done
