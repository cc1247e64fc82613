#!/bin/bash
# DAttn + MSDA iteration: parity suites of both, the DAttn kernel trace and the MSDA C5 lines.
cd "$(dirname "$0")/.."
tag=${1:-it}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msda.py -x -q --timeout 240 --timeout-method thread > gpurun_out/msda_tests_$tag.log 2>&1
rc=$?; tail -2 gpurun_out/msda_tests_$tag.log; grep -E "^FAILED" gpurun_out/msda_tests_$tag.log | head -5
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_dattn_iter.sh $tag || exit $?
timeout -k 10 200 python -u -c "
import sys, json; sys.path[:0] = ['.', 'ir-ads_amd']
import torch, bench
k = bench.msda_rooflines(torch.device('cuda', 0))
for n, v in k.items(): print(n, v['avg_launch_ms'], 'ms', v.get('gather_frac'))
" > gpurun_out/msda_bench_$tag.log 2>&1 || { tail gpurun_out/msda_bench_$tag.log; exit 1; }
cat gpurun_out/msda_bench_$tag.log
