#!/bin/bash
# Round 5: pipelined GEMM variants (5: 256x128 on 8 waves of 64x64, 3 stages; 6: 128x128, 2 stages)
# against the shipped tilings (2, 4) and hipBLASLt at the C2 trunk shapes (bit-exactness vs variant 2,
# time per call); window-attention GPU tests on the packed-conversion build; one bench step with the
# per-workgroup stamp dump (workgroup timelines of every stamped launch).
set -o pipefail
mkdir -p gpurun_out
GEMM_VARIANTS=4,5,6 timeout -k 10 300 python -u scripts/gemm_ab.py --stages 0,1,2,3 > gpurun_out/gemm_ab_r05.log 2>&1 || { echo "gemm_ab failed rc=$?"; tail -30 gpurun_out/gemm_ab_r05.log; exit 1; }
echo gemm_ab ok
timeout -k 10 700 python -u -m pytest tests/test_gpu_swin.py tests/test_gpu_winattn_variants.py tests/test_gpu_dino_detector.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_swin_dino_r05.log 2>&1 || { echo "swin/dino tests failed"; tail -30 gpurun_out/tests_swin_dino_r05.log; exit 1; }
tail -2 gpurun_out/tests_swin_dino_r05.log
IRADS_STAMP_DUMP=gpurun_out/stamps_r05.npz timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_stamps_r05.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_stamps_r05.log; exit 1; }
tail -1 gpurun_out/bench_stamps_r05.log | cut -c1-600
python scripts/stamp_timeline.py gpurun_out/stamps_r05.npz --name winattn_fwd > gpurun_out/stamp_timeline_fwd_r05.txt
python scripts/stamp_timeline.py gpurun_out/stamps_r05.npz --name winattn_bwd > gpurun_out/stamp_timeline_bwd_r05.txt
cat gpurun_out/stamp_timeline_fwd_r05.txt
