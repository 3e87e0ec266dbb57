# GIL switch interval A/B on the RAG bench, alternating (5 ms CPython default vs 1 ms)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/switch2
python -m compileall -q langstream_amd > /dev/null
for sw in "" 1 "" 1 "" 1; do
  LANGSTREAM_SWITCH_MS=$sw timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --also-stream 0 > gpurun_out/switch2/rag_$sw.log 2>&1 || { tail -20 gpurun_out/switch2/rag_$sw.log; exit 1; }
  grep '"metric"' gpurun_out/switch2/rag_$sw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('sw=$sw', r['value'], r['p50_latency_s'])"
done
