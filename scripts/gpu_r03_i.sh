#!/bin/bash
# PMC passes of the window-attention forward / backward (r03 kernels), the MSDA bucket passes with
# quad-aggregated atomics (parity + per-kernel trace), and a bench line with the repeated-launch timer.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
IRADS_PMC_KIND=fwd bash scripts/pmc_winattn_kind.sh r03 || exit $?
IRADS_PMC_KIND=bwd bash scripts/pmc_winattn_kind.sh r03 || exit $?
bash scripts/gpu_msda_iter.sh || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r03i.log 2>&1 || { tail -3 gpurun_out/bench_r03i.log; exit 1; }
tail -1 gpurun_out/bench_r03i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:600], json.dumps(d['roofline_bwd']), json.dumps(d['kernels']['msda_bwd_encoder'])[:300])"
bash scripts/gpu_r03_j.sh
