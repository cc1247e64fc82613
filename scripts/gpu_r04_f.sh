#!/bin/bash
# Round 4: the RCCL capture test (quiesced watchdogs), then the DINO detector product dump in fp64
# for scripts/dino_det_dump.py compare.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_zz_rccl.py -x -v --timeout 240 --timeout-method thread > gpurun_out/rccl_$1.log 2>&1; rc=$?
tail -3 gpurun_out/rccl_$1.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u scripts/dino_det_dump.py product gpurun_out/dino_det_product.npz > gpurun_out/dino_dump_$1.log 2>&1 || { tail -20 gpurun_out/dino_dump_$1.log; exit 1; }
tail -2 gpurun_out/dino_dump_$1.log
exit $rc
