set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "lm_head" > gpurun_out/head_tests.log 2>&1 || { tail -30 gpurun_out/head_tests.log; exit 1; }
tail -1 gpurun_out/head_tests.log
timeout -k 10 300 python -u tools/dgemm_bench.py --only head > gpurun_out/head_bench.log 2>&1 || { tail -20 gpurun_out/head_bench.log; exit 1; }
cat gpurun_out/head_bench.log | grep gemm
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/knnprof -o kp -- python3 tools/engine_bench.py --what knn --rows 1000000 --queries 1024 > gpurun_out/knnprof.log 2>&1 || { tail -20 gpurun_out/knnprof.log; exit 1; }
find gpurun_out/knnprof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/knn_kernel_stats.csv
cut -d, -f1-8 gpurun_out/knn_kernel_stats.csv | head -12
for v in 0 1; do
  LS_DGEMM_HEAD=$v timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eb_head$v.log 2>&1 || exit $?
  echo "LS_DGEMM_HEAD=$v $(tail -1 gpurun_out/eb_head$v.log | cut -c1-260)"
done
