# kNN mid-tile sync A/B (LS_KNN_MIDSYNC), tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4q}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "knn or vector" --timeout 120 --timeout-method thread > gpurun_out/knn_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/knn_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
LS_KNN_MIDSYNC=$v timeout -k 10 300 python -u tools/engine_bench.py --what knn --queries 256,1024,2048 --iters 20 > gpurun_out/knn_bench_mid${v}_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_bench_mid${v}_$TAG.log; exit 1; }
echo "mid=$v $(grep '"knn"' gpurun_out/knn_bench_mid${v}_$TAG.log | python3 -c '
import json,sys
print(" ".join(f"Q{d[\"queries\"]}={d[\"ms\"]}" for d in map(json.loads, sys.stdin)))')"
done
