# r5: the multi-rank code path at world 1 with the per-round kNN load of 8 ranks
# (LS_KNN_REPLICATE=8) and the stage trace, on the prefix-cache tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5o}
LS_STAGE_TRACE=1 LS_BENCH_FORCE_DIST=1 LS_KNN_REPLICATE=8 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --steps 5 --warmup 3 > gpurun_out/knn_w8load_$T.log 2>&1 || { tail -30 gpurun_out/knn_w8load_$T.log; exit 1; }
grep '"metric"' gpurun_out/knn_w8load_$T.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_s'], d['config']['parallelism'], d.get('knn_rounds_per_rank'), d.get('knn_stats_rank0'), d['step_phases_rank0_s'])"
