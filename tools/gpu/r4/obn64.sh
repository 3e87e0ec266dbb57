# o projection on 64-column tiles: kernel + engine tests, then B = 256 decode A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4s}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "decode_gemm or dgemm or routing_at_m_rows or native_executor or graph_decode or norm_deferred or llama" --timeout 300 --timeout-method thread > gpurun_out/obn64_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/obn64_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
LS_DGEMM_O_BN64=$v timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eng_b256_obn64_${v}_$TAG.log 2>&1 || { tail -20 gpurun_out/eng_b256_obn64_${v}_$TAG.log; exit 1; }
echo "o_bn64=$v $(grep -o '"ms_per_decode_step": [0-9.]*' gpurun_out/eng_b256_obn64_${v}_$TAG.log)"
done
