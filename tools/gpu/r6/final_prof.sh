# r6: round-end checks on the current tree (GPU suite, smoke, headline bench with the
# driver's step counts, config 3), then the headline bench's kernel stats under rocprofv3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r6g}
bash tools/gpu/r6/final.sh $T || exit $?
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_prof_$T.log 2>&1 || { tail -30 gpurun_out/bench_prof_$T.log; exit 1; }
tail -1 gpurun_out/bench_prof_$T.log | cut -c1-200
find gpurun_out/prof_$T -type f ! -name '*stats.csv' -delete
find gpurun_out/prof_$T -name '*kernel_stats.csv'
