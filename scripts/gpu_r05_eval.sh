#!/bin/bash
# The detectron2-free vCLR eval path: HIP NMS, post-processing, eval driver; the detector tests beside.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dino_eval.py tests/test_gpu_dino_detector.py -m gpu -v -rfs --timeout 240 --timeout-method thread > gpurun_out/tests_eval_r05.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/tests_eval_r05.log | tail -20; tail -3 gpurun_out/tests_eval_r05.log; exit $rc
