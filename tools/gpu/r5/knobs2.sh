# r5: confirm LS_DGEMM_SPLIT_OUTER=0 (split-K slices of one tile adjacent) and NTST=0 at
# B = 256 and B = 64 (engine_bench), three rounds interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/knobs2_r5ae.log
: > $OUT
for r in 1 2 3; do
  for kv in "X=0" "LS_DGEMM_SPLIT_OUTER=0" "LS_DGEMM_SPLIT_OUTER=0 LS_DGEMM_NTST=0"; do
    for b in 256 64; do
      env $kv timeout -k 10 240 python -u tools/engine_bench.py --what llm --batch $b --prompt 410 --gen 128 --iters 2 > gpurun_out/knob.log 2>&1 || { tail -20 gpurun_out/knob.log; exit 1; }
      echo "$kv B=$b run $r $(grep -o '"ms_per_decode_step": [0-9.]*' gpurun_out/knob.log | tail -1)" | tee -a $OUT
    done
  done
done
