# grouped V-cache layout: full GPU suite, attention / qkv+rope timing, engine decode step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_vl.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_vl.log; [ $rc -eq 0 ] || exit $rc
for args in "--shapes 256x410" "--shapes 256x566 --uniform-lo 265 --sorted"; do
  timeout -k 10 120 python -u tools/attn_bench.py $args --ring 4 --check-all 2>&1 | grep '"B"' | cut -c1-120 || exit 1
done
timeout -k 10 300 python -u tools/dgemm_bench.py --only qkv --rounds 5 > gpurun_out/dg_qkv_vl.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/dg_qkv_vl.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['gemm'], {k:v for k,v in r['us'].items() if k in ('dgemm_bn128_s4','qkvrope_pass')})"
timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eb_vl.log 2>&1 || exit $?
tail -1 gpurun_out/eb_vl.log | cut -c1-300
