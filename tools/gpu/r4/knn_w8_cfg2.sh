# (1) the multi-rank path at world 1 with the per-round kNN load of 8 ranks
#     (LS_KNN_REPLICATE=8: every round searches the gathered queries 8x over), knn_stats logged;
# (2) config 2 (compute-ai-embeddings on Kafka) under the whole-process stack sampler.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LS_BENCH_FORCE_DIST=1 LS_KNN_REPLICATE=8 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/knn_w8load.log 2>&1
rc=$?; grep '"metric"' gpurun_out/knn_w8load.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_s'], d['config']['parallelism'], d.get('knn_rounds_per_rank'), d.get('knn_stats_rank0'))" || tail -30 gpurun_out/knn_w8load.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/stack_sampler.py --every-ms 2 --top 50 -- bench.py --config embed --steps 3 --warmup 1 --batch 2048 > gpurun_out/cfg2_stacks.log 2>&1 || { tail -30 gpurun_out/cfg2_stacks.log; exit 1; }
grep '"metric"' gpurun_out/cfg2_stacks.log | cut -c1-250
