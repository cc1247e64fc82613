#!/bin/bash
# AdamW in 72-tensor launches (optimizer / graph tests), then the bench lines on the final round-3 tree (C3 DeepCrack Swin-B 512^2 batch 4,
# C4 MFNet Swin-L 480x640 with the SB hook); the C2 default line is in r03_bench_t.json.
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_optim.py tests/test_gpu_graph.py > gpurun_out/u_tests.log 2>&1
rc=$?; echo "optim/graph tests rc=$rc"; tail -1 gpurun_out/u_tests.log; [ $rc -ne 0 ] && exit $rc
for w in c2 c3 c4; do
  timeout -k 10 500 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r03u_$w.log 2>&1 || { echo "bench $w failed"; tail -5 gpurun_out/bench_r03u_$w.log; exit 1; }
  tail -1 gpurun_out/bench_r03u_$w.log | cut -c1-300
done
