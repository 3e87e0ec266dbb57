# r5: same-box A/B of this round's last two defaults in the RAG bench: the LM head on the
# ping-pong kernel (LS_HEAD_PP_MIN_T=0 turns it off) and all-nt attention loads
# (LS_ATTN_NT=2: first block cached), two rounds interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/ab_head_attn_r5ai.log
: > $OUT
for r in 1 2; do
  for kv in "X=0" "LS_HEAD_PP_MIN_T=0" "LS_ATTN_NT=2"; do
    env $kv timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
    echo "$kv run $r $(grep '"metric"' gpurun_out/b.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["engine_rank0"]["exec_ms"]["wait"], r["engine_rank0"]["decode_steps"], r["stream_load"]["value"])')" | tee -a $OUT
  done
done
