# Per-CU ingest microbenchmark (LDS-DMA vs VGPR loads, L2 vs HBM, concurrent) + a short
# bench run on the current tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5c}
timeout -k 10 120 tools/bin/ingest_bench > gpurun_out/ingest_$T.log 2>&1 || { cat gpurun_out/ingest_$T.log; exit 1; }
cat gpurun_out/ingest_$T.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_$T.log 2>&1 || { tail -30 gpurun_out/bench_$T.log; exit 1; }
tail -1 gpurun_out/bench_$T.log | cut -c1-400
