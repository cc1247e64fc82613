#!/bin/bash
# Every -m gpu suite in one pytest process (per-test thread timeouts), then smoke().
# Usage: scripts/gpu_all.sh [tag] [pytest -k expression]
cd "$(dirname "$0")/.."
tag=${1:-all}; kexpr=${2:-}
mkdir -p gpurun_out
args=(tests -m gpu -v -rfs --timeout 240 --timeout-method thread)
[ -n "$kexpr" ] && args+=(-k "$kexpr")
NCCL_DEBUG=${NCCL_DEBUG:-WARN} timeout -k 10 ${GPU_ALL_TIMEOUT:-900} python -u -m pytest "${args[@]}" > gpurun_out/tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/tests_$tag.log | grep -v PASSED | tail -20; tail -3 gpurun_out/tests_$tag.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
exit $rc
