#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_drivers.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/drivers_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/drivers_tests.log
exit $rc
