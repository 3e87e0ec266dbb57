set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "knn or qkv_rope or decode_gemm or gemm_prefill" > gpurun_out/knn_rope_tests.log 2>&1 || { tail -30 gpurun_out/knn_rope_tests.log; exit 1; }
tail -2 gpurun_out/knn_rope_tests.log
timeout -k 10 200 python -u tools/engine_bench.py --what knn --rows 1000000 --queries 64,256,1024,2048 > gpurun_out/knn_bench.log 2>&1 || { tail -20 gpurun_out/knn_bench.log; exit 1; }
LS_KNN_Q256_MIN=100000 timeout -k 10 200 python -u tools/engine_bench.py --what knn --rows 1000000 --queries 256,1024,2048 >> gpurun_out/knn_bench.log 2>&1 || { tail -20 gpurun_out/knn_bench.log; exit 1; }
grep knn gpurun_out/knn_bench.log
for v in 0 1; do
  LS_QKV_ROPE=$v timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eb_qkvrope$v.log 2>&1 || exit $?
  echo "LS_QKV_ROPE=$v $(tail -1 gpurun_out/eb_qkvrope$v.log | cut -c1-260)"
done
