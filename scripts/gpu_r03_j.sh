#!/bin/bash
# Where the step's torch glue comes from (current tree): the cast / copy / add audit by bytes and by
# launches, and every aten op with a kernel by bytes.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/cast_audit.py --top 45 > gpurun_out/cast_audit_r03.txt 2>&1 || { tail -5 gpurun_out/cast_audit_r03.txt; exit 1; }
timeout -k 10 300 python -u scripts/cast_audit.py --all-ops --by-site --by-count --top 60 > gpurun_out/op_audit_r03.txt 2>&1 || { tail -5 gpurun_out/op_audit_r03.txt; exit 1; }
head -50 gpurun_out/cast_audit_r03.txt; head -62 gpurun_out/op_audit_r03.txt
