#!/bin/bash
# irads_gemm_nt in the trunk: the fused-stage and GEMM tests, then the bench line with the
# selection table (IRADS_GEMM=table) against hipBLASLt everywhere (IRADS_GEMM=off), interleaved.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_swin_fused.py > gpurun_out/tests_n.log 2>&1 || { tail -30 gpurun_out/tests_n.log; exit 1; }
tail -2 gpurun_out/tests_n.log
for rep in 1 2; do
  for arm in off table; do
    IRADS_GEMM=$arm timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-kernels --no-cpu-baseline > gpurun_out/bench_irgemm_${arm}_$rep.log 2>&1 || { echo "bench $arm failed"; tail -5 gpurun_out/bench_irgemm_${arm}_$rep.log; exit 1; }
    echo "$arm $rep $(tail -1 gpurun_out/bench_irgemm_${arm}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
