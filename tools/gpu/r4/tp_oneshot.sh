# Multi-process one-shot all-reduce and the TP=2 native executor with it, two ranks on cuda:0.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4j}
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_dist_gpu.py tests/test_engine_gpu.py -k "processes_sharing or two_ranks_one_gpu or oneshot" > gpurun_out/tp_oneshot_$T.log 2>&1 || { tail -40 gpurun_out/tp_oneshot_$T.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/tp_oneshot_$T.log
