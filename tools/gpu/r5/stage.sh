# r5: RAG bench with the stage trace (searches + per-thread CPU over each step's front).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5w}
LS_STAGE_TRACE=1 timeout -k 10 500 python -u bench.py > gpurun_out/bench_stage_$T.log 2>&1 || { tail -30 gpurun_out/bench_stage_$T.log; exit 1; }
tail -1 gpurun_out/bench_stage_$T.log | cut -c1-250
