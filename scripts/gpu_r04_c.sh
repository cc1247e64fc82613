#!/bin/bash
# Window-attention forward variants: bit-exact tests, then the A/B timing lab.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_winattn_variants.py -x -q --timeout 120 --timeout-method thread > gpurun_out/winattn_variants_test.log 2>&1; rc=$?
tail -5 gpurun_out/winattn_variants_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/winattn_ab.py > gpurun_out/winattn_ab_$1.log 2>&1 || { echo lab failed; tail -20 gpurun_out/winattn_ab_$1.log; exit 1; }
cat gpurun_out/winattn_ab_$1.log | grep -v "^{\"side" ; grep "^{\"side" gpurun_out/winattn_ab_$1.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['side'],d['shift'],d['variant'],d['us'],d['frac_of_8TBs'])"
