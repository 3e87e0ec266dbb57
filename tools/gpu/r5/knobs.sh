# r5: decode-step knobs at B = 256 (engine_bench), two rounds interleaved:
# default / LS_DGEMM_NTST=0 / LS_DGEMM_SPLIT_OUTER=0 / LS_DGEMM_O_BN64=0 / LS_ATTN_WPP=4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/knobs_r5ad.log
: > $OUT
for r in 1 2; do
  for kv in "X=0" "LS_DGEMM_NTST=0" "LS_DGEMM_SPLIT_OUTER=0" "LS_DGEMM_O_BN64=0" "LS_ATTN_WPP=4"; do
    env $kv timeout -k 10 240 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 --iters 2 > gpurun_out/knob.log 2>&1 || { tail -20 gpurun_out/knob.log; exit 1; }
    echo "$kv run $r $(grep -o '"ms_per_decode_step": [0-9.]*' gpurun_out/knob.log | tail -1)" | tee -a $OUT
  done
done
