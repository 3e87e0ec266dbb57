# kNN pipelined-kernel check + bench at Q=1024/2048, config 2 with out-of-process
# Kafka clients, then the headline bench + timed-window timeline.
# usage: bash tools/gpu/r4/knn_cfg2_bench.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4d}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "knn or vector" --timeout 120 --timeout-method thread > gpurun_out/knn_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/knn_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/engine_bench.py --what knn --queries 64,256,1024,2048 --iters 20 > gpurun_out/knn_bench_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_bench_$TAG.log; exit 1; }
grep -i "knn" gpurun_out/knn_bench_$TAG.log | tail -8
for R in 1 2 4; do
timeout -k 10 400 python -u bench.py --config embed --steps 5 --warmup 1 --batch 2048 --embed-replicas $R > gpurun_out/cfg2_${TAG}_R$R.log 2>&1 || { tail -30 gpurun_out/cfg2_${TAG}_R$R.log; exit 1; }
grep '"metric"' gpurun_out/cfg2_${TAG}_R$R.log | cut -c90-200
done
bash tools/gpu/r3_bench.sh $TAG
