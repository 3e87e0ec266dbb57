# r5: same-box A/B of the LM head on the ping-pong kernel in the RAG bench
# (LS_HEAD_PP_MIN_T=0: the decode GEMM head), three rounds interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/ab_head_r5ak.log
: > $OUT
for r in 1 2 3; do
  for kv in "X=0" "LS_HEAD_PP_MIN_T=0"; do
    env $kv timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
    echo "$kv run $r $(grep '"metric"' gpurun_out/b.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["engine_rank0"]["exec_ms"]["wait"], r["engine_rank0"]["decode_steps"], r["stream_load"]["value"])')" | tee -a $OUT
  done
done
