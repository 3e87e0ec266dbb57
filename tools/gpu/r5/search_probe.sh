set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5l}
timeout -k 10 300 python -u tools/search_latency_probe.py > gpurun_out/search_probe_$T.log 2>&1 || { tail -30 gpurun_out/search_probe_$T.log; exit 1; }
tail -1 gpurun_out/search_probe_$T.log
