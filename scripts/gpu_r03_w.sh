#!/bin/bash
# DAttn proj_k / proj_v as one stacked Linear: DAttn, training-step, determinism, graph and swin tests,
# then the bench line and a kernel trace.
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -v -rfs --timeout 240 --timeout-method thread -m gpu tests/test_gpu_dattn_native.py tests/test_gpu_train_parity.py tests/test_gpu_determinism.py tests/test_gpu_graph.py tests/test_gpu_swin.py > gpurun_out/w_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/w_tests.log | head -8; tail -1 gpurun_out/w_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r03w.log 2>&1 || { echo bench failed; tail gpurun_out/bench_r03w.log; exit 1; }
tail -1 gpurun_out/bench_r03w.log | cut -c1-300
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_r03w --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
f=$(find gpurun_out/prof_r03w -name "*kernel_trace.csv.gz" | head -1); python3 scripts/trace_summary.py "$f" --steps 4 --top 60 > gpurun_out/step_breakdown_r03w.txt 2>&1; head -1 gpurun_out/step_breakdown_r03w.txt
