# r5: config 5's model at world 1 (Llama-3-70B, 140 GB bf16 on one GPU) through the gateway.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r5z}
mkdir -p gpurun_out
timeout -k 10 700 python -u bench.py --config chat --chat-model llama-3-70b --steps 2 --warmup 1 > gpurun_out/cfg5_$T.log 2>&1 || { tail -30 gpurun_out/cfg5_$T.log; exit 1; }
grep '"metric"' gpurun_out/cfg5_$T.log | cut -c1-400
