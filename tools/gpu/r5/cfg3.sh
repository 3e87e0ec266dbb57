# r5: config 3 (Llama-3-8B chat through the websocket gateway, 64 sessions) on the
# current tree, and config 1 (text splitter, CPU) for the record.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r5m}
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --config chat --steps 3 --warmup 1 > gpurun_out/cfg3_$T.log 2>&1 || { tail -30 gpurun_out/cfg3_$T.log; exit 1; }
grep '"metric"' gpurun_out/cfg3_$T.log | cut -c1-400
