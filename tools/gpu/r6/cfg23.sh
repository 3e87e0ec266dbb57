# r6: config 2 (embeddings agent on Kafka, one agent process and the default replicas)
# and config 3 (chat) on the current tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg
timeout -k 10 500 python -u bench.py --config embed --steps 20 --warmup 3 > gpurun_out/cfg/cfg2_r6f.log 2>&1 || { tail -30 gpurun_out/cfg/cfg2_r6f.log; exit 1; }
grep '"metric"' gpurun_out/cfg/cfg2_r6f.log | cut -c1-220
timeout -k 10 500 python -u bench.py --config chat --steps 3 --warmup 1 > gpurun_out/cfg/cfg3_r6f.log 2>&1 || { tail -30 gpurun_out/cfg/cfg3_r6f.log; exit 1; }
grep '"metric"' gpurun_out/cfg/cfg3_r6f.log | cut -c1-220
