# prefill qkv/o/down: hipBLASLt vs gemm_pp over the step sizes the RAG bench produces; config 2 stack samples
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/gemm_prefill_bench.py --ms 3072,4096,5081,6144,7155,8192,9531,11607,12288,12478,13550,16111,16384 --only llama_qkv,llama_o,llama_down --ours --big > gpurun_out/pgemm_m2.log 2>&1 || exit $?
grep '"M"' gpurun_out/pgemm_m2.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['M'], r['gemm'], r['hipblaslt_tflops'], r.get('ours_tflops'), r.get('speedup'))"
bash tools/gpu/r3c_cfg2prof.sh
