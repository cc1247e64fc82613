#!/bin/bash
# Run the -m gpu parity suites file by file on the GPU box.  A plain test failure
# (pytest exit 1) moves on to the next file; any crash / abort / timeout stops the run.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for f in "$@"; do
  name=$(basename "$f" .py)
  timeout -k 10 ${GPU_TEST_TIMEOUT:-600} python -m pytest "$f" -m gpu -q -rf --timeout=300 > gpurun_out/${name}.log 2>&1
  rc=$?
  echo "$f rc=$rc"; tail -3 gpurun_out/${name}.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $f exited with $rc"; exit $rc; fi
done
exit 0
