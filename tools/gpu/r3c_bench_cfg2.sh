# headline bench + timeline, then config 2 at larger steps
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r3_bench.sh ${1:-r3h} || exit $?
bash tools/gpu/r3c_cfg2.sh
timeout -k 10 300 python -u tools/gemm_prefill_bench.py --ms 768,1280,2304,4352,8448,16640 --only llama_qkv,llama_o,llama_down,llama_gate_up --ours --big > gpurun_out/pgemm_midm.log 2>&1 || exit $?
grep '"M"' gpurun_out/pgemm_midm.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['M'], r['gemm'], r['hipblaslt_tflops'], r.get('ours_tflops'), r.get('speedup'))"
