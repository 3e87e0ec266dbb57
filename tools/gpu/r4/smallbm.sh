# 64/128-row decode GEMM tiles: kernel tests, routing test, small-M bench A/B, B = 64 engine.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4k}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "decode_gemm or dgemm or skinny or routing_at_m_rows or native_executor or graph_decode" --timeout 300 --timeout-method thread > gpurun_out/smallbm_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/smallbm_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
LS_DGEMM_SMALL_BM=$v timeout -k 10 300 python -u tools/dgemm_bench.py --ms 5,33,64,100,128 --only qkv,gate_up,down,head --rounds 3 --iters 20 > gpurun_out/dgemm_smallm_bm${v}_$TAG.log 2>&1 || { tail -20 gpurun_out/dgemm_smallm_bm${v}_$TAG.log; exit 1; }
grep -v amdgpu gpurun_out/dgemm_smallm_bm${v}_$TAG.log | python3 -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: continue
    u=d['us']; print('bm$v', d['gemm'], d['M'], 'skinny', u.get('skinny'), 'dgemm', u.get('dgemm_bn128_s0'), 'best', d['best'], u[d['best']])
"
done
for v in 0 1; do
LS_DGEMM_SMALL_BM=$v timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 64 --prompt 410 --gen 128 > gpurun_out/eng_b64_bm${v}_$TAG.log 2>&1 || { tail -20 gpurun_out/eng_b64_bm${v}_$TAG.log; exit 1; }
echo "bm$v $(grep -o '"ms_per_decode_step": [0-9.]*' gpurun_out/eng_b64_bm${v}_$TAG.log)"
done
