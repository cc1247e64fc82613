#!/bin/bash
# Round 5: the phase-interleaved 256x256 GEMM (variant 5) — bit-exactness on every tiling and
# epilogue (test_gpu_gemm.py), time per call against variants 2 / 4 and hipBLASLt at the C2 trunk
# shapes (gemm_ab.py); then one bench step with the per-workgroup stamp dump (workgroup timelines).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_gemm_r05.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/tests_gemm_r05.log; exit 1; }
tail -2 gpurun_out/tests_gemm_r05.log
GEMM_VARIANTS=4,5 timeout -k 10 300 python -u scripts/gemm_ab.py --stages 0,1,2,3 > gpurun_out/gemm_ab_r05b.log 2>&1 || { echo "gemm_ab failed rc=$?"; tail -30 gpurun_out/gemm_ab_r05b.log; exit 1; }
echo gemm_ab ok
IRADS_STAMP_DUMP=gpurun_out/stamps_r05.npz timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-kernels --no-cpu-baseline > gpurun_out/bench_stamps_r05.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_stamps_r05.log; exit 1; }
tail -1 gpurun_out/bench_stamps_r05.log | cut -c1-400
python scripts/stamp_timeline.py gpurun_out/stamps_r05.npz --name winattn_fwd > gpurun_out/stamp_timeline_fwd_r05.txt
python scripts/stamp_timeline.py gpurun_out/stamps_r05.npz --name winattn_bwd > gpurun_out/stamp_timeline_bwd_r05.txt
cat gpurun_out/stamp_timeline_fwd_r05.txt
