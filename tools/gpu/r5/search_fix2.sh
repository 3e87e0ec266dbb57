# r5: vector-store GPU tests, then the RAG bench twice (stage trace on the 2nd) after the
# upsert / search lock-scope changes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5v}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "vector or knn or store or search" > gpurun_out/vs_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/vs_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/bench_${T}_1.log 2>&1 || { tail -30 gpurun_out/bench_${T}_1.log; exit 1; }
tail -1 gpurun_out/bench_${T}_1.log | cut -c1-250
LS_STAGE_TRACE=1 timeout -k 10 500 python -u bench.py > gpurun_out/bench_${T}_2.log 2>&1 || { tail -30 gpurun_out/bench_${T}_2.log; exit 1; }
tail -1 gpurun_out/bench_${T}_2.log | cut -c1-250
