#!/bin/bash
# Round-3 baseline on the restored tree: full -m gpu suite + smoke, bench line, kernel trace,
# then the persistent window-attention forward A/B (IRADS_WINATTN_FWD_PC = workgroups per CU).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/parity
export IRADS_REPORT_DIR=gpurun_out/parity
GPU_ALL_TIMEOUT=1000 bash scripts/gpu_all.sh r03d || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03d.log 2>&1 || { echo bench failed; tail gpurun_out/bench_r03d.log; exit 1; }
tail -1 gpurun_out/bench_r03d.log
PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_r03d --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
IRADS_WINATTN_FWD_PC=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_swin.py tests/test_gpu_swin_fused.py > gpurun_out/pc4_tests.log 2>&1; rc=$?
echo "pc4 tests rc=$rc"; tail -3 gpurun_out/pc4_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for pc in 0 3 4 5; do
  IRADS_WINATTN_FWD_PC=$pc timeout -k 10 200 python -u scripts/winattn_lab.py > gpurun_out/lab_pc$pc.log 2>&1 || exit $?
  echo "pc=$pc"; grep step_avg gpurun_out/lab_pc$pc.log
done
timeout -k 10 200 python -u scripts/msda_bench.py > gpurun_out/msda_bench_r03d.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/msda_bench_r03d.log | cut -c1-200
