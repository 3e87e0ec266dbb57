# r5: kernel stats of the headline RAG bench (rocprofv3 kernel trace, 3 timed steps).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r5am}
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_prof_$T.log 2>&1 || { tail -30 gpurun_out/bench_prof_$T.log; exit 1; }
tail -1 gpurun_out/bench_prof_$T.log | cut -c1-200
find gpurun_out/prof_$T -name '*kernel_stats.csv' | head -3
# keep the summaries only (the whole trace exceeds what gpurun copies back)
find gpurun_out/prof_$T -type f ! -name '*stats.csv' -delete
du -sh gpurun_out/prof_$T
