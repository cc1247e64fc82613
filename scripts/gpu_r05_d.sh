#!/bin/bash
# Round 5: pass-Q lane interleave; stamps on/off A/B kernel traces.
cd "$(dirname "$0")/.."
tag=${1:-r05d}
timeout -k 10 600 python -u -m pytest tests/test_gpu_dattn_native.py tests/test_gpu_determinism.py \
    -m gpu -q -rfs --timeout 300 --timeout-method thread -s > gpurun_out/tests_${tag}.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/tests_${tag}.log | head; tail -1 gpurun_out/tests_${tag}.log
grep -E "^rpe " gpurun_out/tests_${tag}.log | head -4
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for mode in on off; do
  if [ $mode = off ]; then export IRADS_NO_STAMPS=1; fi
  PROFILE_TIMEOUT=300 bash scripts/profile_bench.sh prof_${tag}_$mode --steps 4 --warmup 4 --no-cpu-baseline --profile-only || exit $?
  f=$(find gpurun_out/prof_${tag}_$mode -name "*kernel_trace.csv.gz" | head -1); python3 scripts/trace_summary.py "$f" --steps 4 --match "winattn|dattn_attn" > gpurun_out/step_breakdown_${tag}_$mode.txt 2>&1
  echo "== stamps $mode"; head -1 gpurun_out/step_breakdown_${tag}_$mode.txt; grep -E "winattn|dattn_attn" gpurun_out/step_breakdown_${tag}_$mode.txt | head -7
done
