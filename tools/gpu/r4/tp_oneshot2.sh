# One-shot collectives (bf16 / int64 sums, 32-bit gathers) between processes sharing cuda:0,
# and TP=2 native decode with every collective on them, eager and graph-captured.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4k}
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_dist_gpu.py tests/test_engine_gpu.py -k "processes_sharing or two_ranks_one_gpu or oneshot or tp_path" > gpurun_out/tp_oneshot_$T.log 2>&1 || { tail -40 gpurun_out/tp_oneshot_$T.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/tp_oneshot_$T.log
