# kNN iteration: GPU tests of the store/kNN, bench at Q=64..2048, per-kernel stats at Q=2048.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4g}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "knn or vector" --timeout 120 --timeout-method thread > gpurun_out/knn_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/knn_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/engine_bench.py --what knn --queries 64,256,1024,2048 --iters 20 > gpurun_out/knn_bench_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_bench_$TAG.log; exit 1; }
grep '"knn"' gpurun_out/knn_bench_$TAG.log
bash tools/gpu/r4/knn_prof.sh $TAG | head -5
