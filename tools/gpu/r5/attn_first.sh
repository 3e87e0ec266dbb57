# r5: decode attention with each sequence's first KV block loaded cached (shared
# template-prefix blocks) vs every KV load non-temporal (LS_ATTN_NT=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5i}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 240 --timeout-method thread \
  -k "attention or attn or decode or prefix" > gpurun_out/attn_tests_$T.log 2>&1 || { tail -30 gpurun_out/attn_tests_$T.log; exit 1; }
tail -2 gpurun_out/attn_tests_$T.log
timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_first_$T.log 2>&1 || { tail -30 gpurun_out/bench_first_$T.log; exit 1; }
tail -1 gpurun_out/bench_first_$T.log | cut -c1-250
LS_ATTN_NT=1 timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_allnt_$T.log 2>&1 || { tail -30 gpurun_out/bench_allnt_$T.log; exit 1; }
tail -1 gpurun_out/bench_allnt_$T.log | cut -c1-250
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/tl_$T -o tl -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_prof_$T.log 2>&1 || { tail -20 gpurun_out/bench_prof_$T.log; exit 1; }
DB=$(find gpurun_out/tl_$T -name '*.db' | head -1)
MS=$(grep '"metric"' gpurun_out/bench_prof_$T.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*3/1000)')
python3 tools/timeline_window.py $DB --window-s $MS --top 40 > gpurun_out/timeline_$T.txt
head -16 gpurun_out/timeline_$T.txt
rm -f $DB
