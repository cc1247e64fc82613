#!/bin/bash
# The re-tuned GEMM table: its entries, the C2 table-vs-off step and the training-step pins, then the bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/parity_r05t
export IRADS_REPORT_DIR=gpurun_out/parity_r05t
timeout -k 10 800 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_gemm_step.py tests/test_gpu_train_parity.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/tests_table_r05.log 2>&1
rc=$?; tail -3 gpurun_out/tests_table_r05.log; grep -E "FAILED|ERROR" gpurun_out/tests_table_r05.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r05t.json 2> gpurun_out/bench_r05t.err || { echo bench failed; tail gpurun_out/bench_r05t.err; exit 1; }
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/bench_r05t.json").read().strip().splitlines()[-1])
print(r["value"], r["ms_per_step"], "fwd", r["roofline"]["frac"], "bwd", r["roofline_bwd"]["frac"], "gemm", r.get("roofline_gemm", {}).get("frac"))
PY
