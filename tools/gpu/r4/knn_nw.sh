# kNN filter with 4 waves x 64 queries (LS_KNN_NW=4) vs 8 waves x 32: tests under both, bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4v}
mkdir -p gpurun_out
for v in 4 8; do
LS_KNN_NW=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "knn or vector" --timeout 120 --timeout-method thread > gpurun_out/knn_tests_nw${v}_$TAG.log 2>&1
rc=$?; echo "nw=$v $(tail -1 gpurun_out/knn_tests_nw${v}_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in 4 8 4 8; do
LS_KNN_NW=$v timeout -k 10 300 python -u tools/engine_bench.py --what knn --queries 256,1024,2048 --iters 20 > gpurun_out/knn_bench_nw${v}_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_bench_nw${v}_$TAG.log; exit 1; }
echo "nw=$v $(grep '"knn"' gpurun_out/knn_bench_nw${v}_$TAG.log | tr '\n' ' ' | sed 's/"test": "knn", "rows": 1000000, //g')"
done
