# Round-3 headline run: bench.py (config 4, defaults: persistence on), then the same bench
# under rocprofv3 --kernel-trace and a timed-window breakdown.  usage: bash tools/gpu/r3_bench.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
grep '"metric"' gpurun_out/bench_$TAG.log | cut -c1-600
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/tl_$TAG -o tl -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_prof_$TAG.log 2>&1 || exit $?
DB=$(ls gpurun_out/tl_$TAG/*/tl*.db 2>/dev/null | head -1)
[ -z "$DB" ] && DB=$(find gpurun_out/tl_$TAG -name '*.db' | head -1)
MS=$(grep '"metric"' gpurun_out/bench_prof_$TAG.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*3/1000)')
python3 tools/timeline_window.py $DB --window-s $MS --top 40 > gpurun_out/timeline_$TAG.txt
head -20 gpurun_out/timeline_$TAG.txt
rm -f $DB
