# r5: LM-head tile width at B = 256 (engine_bench): LS_DGEMM_HEAD_BN 128 (default) vs 256,
# three rounds interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/knobs3_r5af.log
: > $OUT
for r in 1 2 3; do
  for kv in "X=0" "LS_DGEMM_HEAD_BN=256"; do
    env $kv timeout -k 10 240 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 --iters 2 > gpurun_out/knob.log 2>&1 || { tail -20 gpurun_out/knob.log; exit 1; }
    echo "$kv run $r $(grep -o '"ms_per_decode_step": [0-9.]*' gpurun_out/knob.log | tail -1)" | tee -a $OUT
  done
done
timeout -k 10 300 python -u tools/dgemm_bench.py --ms 256 --only head --rounds 5 --iters 10 > gpurun_out/head_r5af.log 2>&1 || { tail -20 gpurun_out/head_r5af.log; exit 1; }
grep '^{' gpurun_out/head_r5af.log | cut -c1-300
