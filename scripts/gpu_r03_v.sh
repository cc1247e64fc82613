#!/bin/bash
# Final tree: the full -m gpu suite and smoke() (bench lines in r03_bench_u_*.json).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/parity
export IRADS_REPORT_DIR=gpurun_out/parity
GPU_ALL_TIMEOUT=1000 bash scripts/gpu_all.sh r03v
