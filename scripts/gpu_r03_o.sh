#!/bin/bash
# Native AdamW (irads_adamw) and the RCCL capture drain: optimizer parity, graph / driver / DP tests,
# the overlapped-exchange capture test twice, then the default bench line.
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -rfs --timeout 240 --timeout-method thread -m gpu tests/test_gpu_optim.py tests/test_gpu_graph.py tests/test_gpu_drivers.py tests/test_gpu_zz_rccl.py > gpurun_out/o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/o_tests.log | head -8; tail -1 gpurun_out/o_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -m pytest -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_zz_rccl.py > gpurun_out/o_rccl2.log 2>&1
rc=$?; echo "rccl rerun rc=$rc"; tail -1 gpurun_out/o_rccl2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03o.log 2>&1 || { echo bench failed; tail gpurun_out/bench_r03o.log; exit 1; }
tail -1 gpurun_out/bench_r03o.log | cut -c1-400
