# decode GEMM K-walk rotation A/B (LS_DGEMM_KROT read per launch, interleaved in one process)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LS_DGEMM_KROT=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests_krot.log 2>&1
rc=$?; tail -2 gpurun_out/dg_tests_krot.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dgemm_bench.py --only qkv,o,gate_up,down --rounds 5 --env-ab LS_DGEMM_KROT > gpurun_out/dg_krot.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/dg_krot.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['gemm'], {k:v for k,v in r['us'].items()})"
