# prefill chunk (engine max-prefill-tokens) A/B on the RAG bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 16384 32768 16384 32768 24576; do
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --prefill-chunk $c > gpurun_out/chunk_$c.log 2>&1 || { tail -20 gpurun_out/chunk_$c.log; exit 1; }
  grep '"metric"' gpurun_out/chunk_$c.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('chunk $c', r['value'], r['p50_latency_s'], r['engine_rank0']['mixed_steps'], r['engine_rank0']['decode_steps'])"
done
