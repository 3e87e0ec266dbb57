# kNN filter priority A/B (LS_KNN_PRIO 0 / 1 / 2), tests under the winner later.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4x}
mkdir -p gpurun_out
for v in 0 1 2 0 1 2; do
LS_KNN_PRIO=$v timeout -k 10 300 python -u tools/engine_bench.py --what knn --queries 256,1024,2048 --iters 20 > gpurun_out/knn_bench_prio${v}_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_bench_prio${v}_$TAG.log; exit 1; }
echo "prio=$v $(grep '"knn"' gpurun_out/knn_bench_prio${v}_$TAG.log | tr '\n' ' ' | sed 's/"test": "knn", "rows": 1000000, //g')"
done
