#!/bin/bash
# Native AdamW parity, then the default bench line (the graph / driver / RCCL tests passed in r03o).
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v -rfs --timeout 240 --timeout-method thread -m gpu tests/test_gpu_optim.py > gpurun_out/q_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|Mismatch|Greatest" gpurun_out/q_tests.log | head -8; tail -1 gpurun_out/q_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03q.log 2>&1 || { echo bench failed; tail gpurun_out/bench_r03q.log; exit 1; }
tail -1 gpurun_out/bench_r03q.log | cut -c1-400
