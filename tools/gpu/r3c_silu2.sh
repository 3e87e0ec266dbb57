# BN=256 gate_up with loader waves (buffer-resource DMA sources): tests + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm or tp8" -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests_s2.log 2>&1
rc=$?; tail -3 gpurun_out/dg_tests_s2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dgemm_bench.py --only gate_up,qkv,o,down --rounds 5 > gpurun_out/dg_s2.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/dg_s2.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['gemm'], {k:v for k,v in r['us'].items() if 'bn256' not in k}, r['err_flag'])"
