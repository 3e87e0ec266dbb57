# r5: prefill split-K for under-filled grids (tests + mid-M timings with and without it),
# prefix-cache shared blocks in the engine tests and the RAG bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5g}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v --timeout 240 --timeout-method thread \
  -k "prefill_pingpong or gemm_prefill_llama or prefix_cache or native_executor_matches or chunked_prefill" > gpurun_out/splitk_tests_$T.log 2>&1 \
  || { tail -40 gpurun_out/splitk_tests_$T.log; exit 1; }
tail -2 gpurun_out/splitk_tests_$T.log
for v in 1 0; do
  LS_PGEMM_SPLITK=$v timeout -k 10 300 python -u tools/gemm_prefill_bench.py --ms 1024,1536,2048,3072 --only llama_o,llama_down,llama_qkv --ours --big > gpurun_out/pgemm_midm_split${v}_$T.log 2>&1 || { tail -20 gpurun_out/pgemm_midm_split${v}_$T.log; exit 1; }
  echo "splitk=$v"; grep -v amdgpu gpurun_out/pgemm_midm_split${v}_$T.log | cut -c1-200
done
LS_PGEMM_SPLITK_MIN_K=4096 timeout -k 10 300 python -u tools/gemm_prefill_bench.py --ms 1024,2048 --only llama_o,llama_qkv --ours --big > gpurun_out/pgemm_midm_splitk4096_$T.log 2>&1 || { tail -20 gpurun_out/pgemm_midm_splitk4096_$T.log; exit 1; }
echo "splitk min_k=4096"; grep -v amdgpu gpurun_out/pgemm_midm_splitk4096_$T.log | cut -c1-200
timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_$T.log 2>&1 || { tail -30 gpurun_out/bench_$T.log; exit 1; }
tail -1 gpurun_out/bench_$T.log | cut -c1-250
