#!/bin/bash
# Round 5: DINO detector tests (forward_student + full training forward) and the C5 detector step line.
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest tests/test_gpu_dino_detector.py -m gpu -v -rfs --timeout 300 --timeout-method thread -s > gpurun_out/tests_dino_r05.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "PASSED|FAILED|ERROR|total .* vs|  !" gpurun_out/tests_dino_r05.log | head -30
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python -u -c "
import sys, json, torch
sys.path.insert(0, 'ir-ads_amd'); sys.argv = ['bench.py']
import bench
print(json.dumps(bench.dino_detector_line(torch.device('cuda', 0))))
" > gpurun_out/dino_det_line_r05.log 2>&1; echo "line rc=$?"; tail -3 gpurun_out/dino_det_line_r05.log
