# r5: engine GPU tests + the RAG bench twice on the current tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5ah}
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/engine_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/engine_tests_$T.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_${T}_$i.log 2>&1 || { tail -30 gpurun_out/bench_${T}_$i.log; exit 1; }
  tail -1 gpurun_out/bench_${T}_$i.log | cut -c1-200
done
