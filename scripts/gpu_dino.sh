cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dino.py -v -x --timeout 240 --timeout-method thread > gpurun_out/dino_tests.log 2>&1; rc=$?
tail -15 gpurun_out/dino_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/dino_bench.py > gpurun_out/dino_bench.json 2> gpurun_out/dino_bench.err || { tail -20 gpurun_out/dino_bench.err; exit 1; }
cat gpurun_out/dino_bench.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['dino_transformer_c5'])"
export TMPDIR=/tmp
DINO_REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dino -o run -- python3 scripts/dino_bench.py > gpurun_out/prof_dino.log 2>&1; echo prof rc=$?
find gpurun_out/prof_dino -name '*kernel_trace.csv' -exec gzip -f {} \;
exit $rc
