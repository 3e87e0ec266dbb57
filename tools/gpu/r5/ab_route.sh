# r5: RAG bench with the prefix cache -- prefill plain GEMMs on the hand-written kernel
# (default) vs routed per M to hipBLASLt where faster (LS_PGEMM=route), then the default's
# kernel timeline of the timed window.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5f}
timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_def_$T.log 2>&1 || { tail -30 gpurun_out/bench_def_$T.log; exit 1; }
tail -1 gpurun_out/bench_def_$T.log | cut -c1-250
LS_PGEMM=route timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_route_$T.log 2>&1 || { tail -30 gpurun_out/bench_route_$T.log; exit 1; }
tail -1 gpurun_out/bench_route_$T.log | cut -c1-250
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/tl_$T -o tl -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_prof_$T.log 2>&1 || { tail -20 gpurun_out/bench_prof_$T.log; exit 1; }
DB=$(find gpurun_out/tl_$T -name '*.db' | head -1)
MS=$(grep '"metric"' gpurun_out/bench_prof_$T.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*3/1000)')
python3 tools/timeline_window.py $DB --window-s $MS --top 40 > gpurun_out/timeline_$T.txt
head -14 gpurun_out/timeline_$T.txt
rm -f $DB
