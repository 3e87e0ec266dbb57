# decode GEMM spread-DMA A/B (BN = 256 launches), ragged attention sensitivity, bench prompt lengths
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dg_tests.log; [ $rc -eq 0 ] || exit $rc
LS_DGEMM_SPREAD=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests_sp.log 2>&1
rc=$?; tail -2 gpurun_out/dg_tests_sp.log; [ $rc -eq 0 ] || exit $rc
for sp in 0 1; do
  LS_DGEMM_SPREAD=$sp timeout -k 10 300 python -u tools/dgemm_bench.py --only gate_up,qkv,o,down --rounds 5 > gpurun_out/dg_sp$sp.log 2>&1 || exit $?
  echo "SPREAD=$sp"; grep -v amdgpu.ids gpurun_out/dg_sp$sp.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['gemm'], {k:v for k,v in r['us'].items()}, r['rel_err'].get('dgemm_s2', ''))"
done
for rg in 0.3 0.5; do
  timeout -k 10 120 python -u tools/attn_bench.py --shapes 256x410 --ragged $rg --ring 4 >> gpurun_out/attn_rg.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/attn_rg.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_pl.log 2>&1 || exit $?
grep '"metric"' gpurun_out/bench_pl.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['prompt_len_pcts_rank0'])"
