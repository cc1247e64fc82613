#!/bin/bash
# Decoder-shape MSDA backward: the tiled bucket walk vs the cell walk (IRADS_MSDA_WALK), twice each.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for mode in cell bucket cell bucket; do
  IRADS_MSDA_WALK=$mode timeout -k 10 120 python -u scripts/msda_bench.py > gpurun_out/msda_dec_$mode.log 2>&1 || { echo "$mode failed"; tail -5 gpurun_out/msda_dec_$mode.log; exit 1; }
  echo "== $mode"; grep -E "^msda_bwd" gpurun_out/msda_dec_$mode.log | python3 -c "
import sys, json
for l in sys.stdin:
    k, v = l.split(' ', 1); print(k, json.loads(v)['avg_launch_ms'])"
done
