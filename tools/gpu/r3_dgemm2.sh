set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dgemm_bench.py --ablate --only qkv,down --rounds 5 > gpurun_out/dg_abl.log 2>&1 || exit $?
cat gpurun_out/dg_abl.log
timeout -k 10 300 python -u tools/dgemm_bench.py --rounds 5 > gpurun_out/dg_bench.log 2>&1 || exit $?
cat gpurun_out/dg_bench.log
