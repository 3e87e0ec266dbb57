# r5: the LM head on the ping-pong kernel with an f32 epilogue -- kernel tests, isolated
# timing at M = 256 (vs the decode GEMM), and the B = 256 decode step with / without it.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "f32_output or lm_head or f32_head" > gpurun_out/head_tests_r5ag.log 2>&1
rc=$?; tail -3 gpurun_out/head_tests_r5ag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u - > gpurun_out/head_pp_r5ag.log 2>&1 <<'PY' || { tail -20 gpurun_out/head_pp_r5ag.log; exit 1; }
import torch, json
from langstream_amd import ops
h = ops.hip()
for M in (129, 192, 256):
    x = torch.randn(M, 4096, device="cuda").to(torch.bfloat16)
    ws = [(torch.randn(128256, 4096, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(2)]
    out = torch.empty(M, 128256, device="cuda", dtype=torch.float32)
    def t(fn, n=20):
        for i in range(3): fn(i)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); s.record()
        for i in range(n): fn(i)
        e.record(); torch.cuda.synchronize()
        return round(s.elapsed_time(e) * 1000 / n, 1)
    r = {"M": M, "pp_f32_us": t(lambda i: h.gemm_prefill_f32(out, x, ws[i % 2])),
         "dgemm_f32_us": t(lambda i: h.decode_gemm_f32(out, x, ws[i % 2], 128))}
    print(json.dumps(r), flush=True)
PY
cat gpurun_out/head_pp_r5ag.log | grep '^{'
for r in 1 2; do for v in 129 0; do
  LS_HEAD_PP_MIN_T=$v timeout -k 10 240 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 --iters 2 > gpurun_out/knob.log 2>&1 || { tail -20 gpurun_out/knob.log; exit 1; }
  echo "HEAD_PP_MIN_T=$v run $r $(grep -o '"ms_per_decode_step": [0-9.]*' gpurun_out/knob.log | tail -1)" | tee -a gpurun_out/head_pp_r5ag.log
done; done
