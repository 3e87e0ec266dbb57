# fused qkv split-K head exchange: kernel tests + timing vs the separate reduction pass
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests_qkv.log 2>&1
rc=$?; tail -3 gpurun_out/dg_tests_qkv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dgemm_bench.py --only qkv --rounds 7 > gpurun_out/dg_qkv.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/dg_qkv.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['gemm'], r['us'], r['err_flag'])"
timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eb_qkv1.log 2>&1 || exit $?
tail -1 gpurun_out/eb_qkv1.log | cut -c1-400
LS_QKV_FUSED=0 timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eb_qkv0.log 2>&1 || exit $?
tail -1 gpurun_out/eb_qkv0.log | cut -c1-400
