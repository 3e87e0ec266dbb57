# bench.py with the driver's round-3 step counts (20 timed after 5 warmup).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4w}
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$T.log 2>&1 || { tail -20 gpurun_out/bench20_$T.log; exit 1; }
grep '"metric"' gpurun_out/bench20_$T.log | cut -c1-400
