# 8 vs 4 loader waves in the decode GEMM (LS_DGEMM_LD8 per launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LS_DGEMM_LD8=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests_ld8.log 2>&1
rc=$?; tail -2 gpurun_out/dg_tests_ld8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dgemm_bench.py --only gate_up,qkv,o,down --rounds 5 --env-ab LS_DGEMM_LD8 > gpurun_out/dg_ld8.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/dg_ld8.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['gemm'], {k:v for k,v in r['us'].items() if 'bn256' not in k and 'dgemm' in k})"
