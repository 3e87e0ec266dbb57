set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 420 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_dist_gpu.py -k "oneshot" -x -q --timeout 120 --timeout-method thread > gpurun_out/ar_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ar_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dgemm_bench.py > gpurun_out/dg_bench.log 2>&1 || exit $?
cat gpurun_out/dg_bench.log
LS_DGEMM=0 timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eb_dg0.log 2>&1 || exit $?
tail -1 gpurun_out/eb_dg0.log | cut -c1-400
timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eb_dg1.log 2>&1 || exit $?
tail -1 gpurun_out/eb_dg1.log | cut -c1-400
