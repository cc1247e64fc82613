#!/bin/bash
# Weight gradients on a side stream: the training-step / graph / determinism tests with it on, then the
# default bench step with IRADS_SIDE_STREAM=0 and without, twice (interleaved).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_parity.py tests/test_gpu_graph.py tests/test_gpu_determinism.py tests/test_gpu_gemm_step.py \
    -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/tests_side.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_side.log; exit 1; }
tail -2 gpurun_out/tests_side.log
for mode in off on off2 on2; do
  case $mode in off*) export IRADS_SIDE_STREAM=0;; *) unset IRADS_SIDE_STREAM;; esac
  timeout -k 10 400 python -u bench.py --no-kernels --no-cpu-baseline --steps 50 > gpurun_out/bench_side_$mode.json 2> gpurun_out/bench_side_$mode.err || { echo "bench $mode failed"; tail -5 gpurun_out/bench_side_$mode.err; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/bench_side_$mode.json').read().strip().splitlines()[-1]); print('$mode', r['value'], r['ms_per_step'])"
done
