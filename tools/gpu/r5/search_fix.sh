# r5: RAG bench (config 4) after the local-search restructure, twice (stage trace on the 2nd).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5p}
timeout -k 10 500 python -u bench.py > gpurun_out/bench_${T}_1.log 2>&1 || { tail -30 gpurun_out/bench_${T}_1.log; exit 1; }
tail -1 gpurun_out/bench_${T}_1.log | cut -c1-300
LS_STAGE_TRACE=1 timeout -k 10 500 python -u bench.py > gpurun_out/bench_${T}_2.log 2>&1 || { tail -30 gpurun_out/bench_${T}_2.log; exit 1; }
tail -1 gpurun_out/bench_${T}_2.log | cut -c1-300
