# Round 4: norm-deferred decode layer -- kernel tests, the whole GPU suite, the engine A/B
# (LS_DGEMM_FUSED 1 vs 0) at B = 256, the prefill GEMM epilogue A/B, and the decode GEMM
# against hipBLASLt at 5..128 rows (the rows the runner now sends to it).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "combine or silu_r or rms_prep" > gpurun_out/fused_kernels.log 2>&1
rc=$?; tail -5 gpurun_out/fused_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r4b.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_r4b.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  LS_DGEMM_FUSED=$f timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eng_fused$f.log 2>&1 || { tail -20 gpurun_out/eng_fused$f.log; exit 1; }
  echo "fused=$f $(grep -v amdgpu.ids gpurun_out/eng_fused$f.log | tail -1 | cut -c1-400)"
done
timeout -k 10 300 python -u tools/pgemm_ab.py --ms 4096,16384 --variants 1,3,4 --rounds 5 > gpurun_out/pp_epi.log 2>&1 || { tail -20 gpurun_out/pp_epi.log; exit 1; }
grep -v amdgpu gpurun_out/pp_epi.log
timeout -k 10 300 python -u tools/dgemm_bench.py --ms 5,33,64,100,128 --only qkv,gate_up,down,head --rounds 5 --iters 20 > gpurun_out/dgemm_smallm.log 2>&1 || { tail -20 gpurun_out/dgemm_smallm.log; exit 1; }
grep -v amdgpu gpurun_out/dgemm_smallm.log | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['gemm'], d['M'], d['us'], d['best'])"
