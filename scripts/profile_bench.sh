#!/bin/bash
# Kernel-trace profile of a short bench.py run on the GPU box.
#   bash scripts/profile_bench.sh <tag> [bench args...]
# Writes gpurun_out/<tag>/run_kernel_stats.csv (+ gzipped trace) and gpurun_out/<tag>.log.
# The raw trace is compressed and anything else large is dropped so that gpurun_out/
# stays under gpurun's 64 MiB copy-back limit.
cd "$(dirname "$0")/.."
tag=$1; shift
out=gpurun_out/$tag
rm -rf "$out"; mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 ${PROFILE_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run \
    -- python3 bench.py "$@" > gpurun_out/$tag.log 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
find "$out" -name '*kernel_trace.csv' -exec gzip -f {} \;
find "$out" -type f \( -name '*.db' -o -size +45M \) -print -delete
du -sh gpurun_out
exit $rc
