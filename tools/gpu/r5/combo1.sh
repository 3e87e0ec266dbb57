# r5: prefix-cache engine tests + RAG bench (prefix cache on), config-2 single process
# (bulk host path), decode GEMM row-block A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5e}
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 240 --timeout-method thread \
  -k "prefix_cache or native_executor_matches or graph_decode or chunked_prefill" > gpurun_out/engine_tests_$T.log 2>&1 \
  || { tail -40 gpurun_out/engine_tests_$T.log; exit 1; }
tail -3 gpurun_out/engine_tests_$T.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_$T.log 2>&1 || { tail -30 gpurun_out/bench_$T.log; exit 1; }
tail -1 gpurun_out/bench_$T.log | cut -c1-300
timeout -k 10 400 python -u bench.py --config embed --steps 5 --warmup 1 --batch 2048 --embed-replicas 1 > gpurun_out/cfg2_${T}_R1.log 2>&1 || { tail -30 gpurun_out/cfg2_${T}_R1.log; exit 1; }
tail -1 gpurun_out/cfg2_${T}_R1.log | cut -c1-300
timeout -k 10 300 python -u tools/dgemm_bench.py --ms 256 --only qkv,gate_up --rounds 5 > gpurun_out/rowblk_$T.log 2>&1 || { tail -30 gpurun_out/rowblk_$T.log; exit 1; }
cut -c1-700 gpurun_out/rowblk_$T.log
