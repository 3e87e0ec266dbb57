# kNN interleaved read/MFMA variant (LS_KNN_ILV=1): tests, then A/B incl. priority.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4y}
mkdir -p gpurun_out
LS_KNN_ILV=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "knn or vector" --timeout 120 --timeout-method thread > gpurun_out/knn_tests_ilv_$TAG.log 2>&1
rc=$?; echo "ilv tests $(tail -1 gpurun_out/knn_tests_ilv_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
for cfg in "0 0" "1 0" "1 2" "0 0" "1 0" "1 2"; do
set -- $cfg
LS_KNN_ILV=$1 LS_KNN_PRIO=$2 timeout -k 10 300 python -u tools/engine_bench.py --what knn --queries 256,1024,2048 --iters 20 > gpurun_out/knn_bench_ilv$1_p$2_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_bench_ilv$1_p$2_$TAG.log; exit 1; }
echo "ilv=$1 prio=$2 $(grep '"knn"' gpurun_out/knn_bench_ilv$1_p$2_$TAG.log | tr '\n' ' ' | sed 's/"test": "knn", "rows": 1000000, //g')"
done
