# bench.py defaults (config 4, 3 timed steps after 1 warmup) on the tree as it is.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4y}
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$T.log 2>&1 || { tail -20 gpurun_out/bench_$T.log; exit 1; }
grep '"metric"' gpurun_out/bench_$T.log | cut -c1-300
