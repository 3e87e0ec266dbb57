# Round 5: decode-GEMM fp32 tests at 5..256 rows with the launch census, the one-shot
# routing fallback, kNN, then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5a}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "decode_gemm" > gpurun_out/dgemm_tests_$T.log 2>&1 || { tail -30 gpurun_out/dgemm_tests_$T.log; exit 1; }
tail -2 gpurun_out/dgemm_tests_$T.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/dist_tests_$T.log 2>&1 || { tail -30 gpurun_out/dist_tests_$T.log; exit 1; }
tail -2 gpurun_out/dist_tests_$T.log
