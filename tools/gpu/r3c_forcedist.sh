# the multi-rank code path at world 1 (torchrun, RCCL default group, sharded-kNN service, shm topics)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LS_BENCH_FORCE_DIST=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/forcedist_r3c.log 2>&1
rc=$?; grep '"metric"' gpurun_out/forcedist_r3c.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_s'], d['config']['parallelism'], d.get('knn_rounds_per_rank'), d.get('knn_stats_rank0'))" || tail -30 gpurun_out/forcedist_r3c.log; exit $rc
