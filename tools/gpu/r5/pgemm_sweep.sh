# r5: prefill ping-pong GEMM tile-order knobs at the RAG bench's chunk size (M = 12288):
# LS_PGEMM_GROUP (M-tiles per group) x LS_PGEMM_SPREAD, one process per setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5an}
for g in 8 4 16; do for sp in 1 0; do
  echo "== GROUP=$g SPREAD=$sp" >> gpurun_out/pgemm_sweep_$T.log
  LS_PGEMM_GROUP=$g LS_PGEMM_SPREAD=$sp timeout -k 10 240 python -u tools/gemm_prefill_bench.py --ms 12288 \
    --only llama_qkv,llama_o,llama_gate_up,llama_down --ours >> gpurun_out/pgemm_sweep_$T.log 2>&1 || exit 1
done; done
grep -c "" gpurun_out/pgemm_sweep_$T.log
