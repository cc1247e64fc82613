#!/bin/bash
# MSDA gather A/B: KC = 8 (default) against KC = 4 (IRADS_MSDA_KC4) grad_out loads per sub-chunk.
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
summ() {
python3 - "$1" <<'PY'
import csv, glob, sys, collections
t = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(t)):
    if "msda" in r["Kernel_Name"]:
        agg[r["Kernel_Name"].replace("(anonymous namespace)::", "")[:48]].append(
            (int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
for k, v in sorted(agg.items()):
    v.sort(); h = len(v) // 2
    enc, dec = [d for _, d in v[:h]], [d for _, d in v[h:]]
    print("%-48s enc %.1f us  dec %.1f us  (n=%d)" % (k, sum(enc) / max(1, len(enc)), sum(dec) / max(1, len(dec)), len(v)))
PY
find "$1" -name "*trace.csv" -delete
}
for v in 8 4; do
  rm -rf gpurun_out/pm$v
  if [ $v = 4 ]; then export IRADS_MSDA_KC4=1; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pm$v -o run -- python3 scripts/msda_bench.py > gpurun_out/pm$v.log 2>&1 || exit 1
  echo "== KC=$v"; grep -E "bwd_encoder|bwd_decoder" gpurun_out/pm$v.log | cut -c1-100
  summ gpurun_out/pm$v
done
