#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_swin.py tests/test_gpu_drivers.py -m gpu -q -k "lightsb or sb_hook" --timeout 200 --timeout-method thread > gpurun_out/sb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/sb_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --workload c4 --steps 20 --warmup 5 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "c4 bench failed"; tail -5 gpurun_out/bench_c4.err; exit 1; }
tail -1 gpurun_out/bench_c4.json | cut -c1-400
