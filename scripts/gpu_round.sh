set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_tests.sh tests/test_gpu_msda.py tests/test_gpu_swin.py tests/test_gpu_seghead.py || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
PROFILE_TIMEOUT=400 bash scripts/profile_bench.sh prof1 --steps 6 --warmup 4 --no-cpu-baseline --profile-only
