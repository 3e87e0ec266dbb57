# kNN default path check: all GPU kNN / vector tests, the bench, the ablations.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4z}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "knn or vector" --timeout 120 --timeout-method thread > gpurun_out/knn_tests_$TAG.log 2>&1
rc=$?; echo "tests $(tail -1 gpurun_out/knn_tests_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/engine_bench.py --what knn --queries 64,256,1024,2048 --iters 20 > gpurun_out/knn_bench_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_bench_$TAG.log; exit 1; }
grep '"knn"' gpurun_out/knn_bench_$TAG.log
bash tools/gpu/r4/knn_abl.sh $TAG
