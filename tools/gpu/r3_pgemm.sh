set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_prefill" > gpurun_out/pgemm_tests.log 2>&1 || { tail -30 gpurun_out/pgemm_tests.log; exit 1; }
tail -3 gpurun_out/pgemm_tests.log
timeout -k 10 400 python -u tools/pgemm_ab.py "$@" > gpurun_out/pgemm_ab.log 2>&1 || { tail -20 gpurun_out/pgemm_ab.log; exit 1; }
cat gpurun_out/pgemm_ab.log
