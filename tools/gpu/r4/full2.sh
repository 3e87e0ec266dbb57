# Whole-tree GPU check: pytest -m gpu, smoke(), headline bench + timeline, W=8 kNN load,
# config 2 at the bench defaults.  usage: bash tools/gpu/r4/full2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4n}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
bash tools/gpu/r3_bench.sh $TAG || exit $?
LS_BENCH_FORCE_DIST=1 LS_KNN_REPLICATE=8 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/knn_w8load_$TAG.log 2>&1 || { tail -30 gpurun_out/knn_w8load_$TAG.log; exit 1; }
grep '"metric"' gpurun_out/knn_w8load_$TAG.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('w8load', d['value'], d['p50_latency_s'], d.get('knn_stats_rank0'))"
timeout -k 10 400 python -u bench.py --config embed --steps 5 --warmup 1 --batch 2048 > gpurun_out/cfg2_$TAG.log 2>&1 || { tail -30 gpurun_out/cfg2_$TAG.log; exit 1; }
grep '"metric"' gpurun_out/cfg2_$TAG.log | cut -c90-220
