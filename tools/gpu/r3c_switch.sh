# GIL switch interval A/B (LANGSTREAM_SWITCH_MS) on config 2 and the RAG bench; crc GIL threshold raised
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for sw in "" 1 "" 1; do
  LANGSTREAM_SWITCH_MS=$sw timeout -k 10 300 python -u bench.py --config embed --batch 2048 --steps 3 --warmup 1 > gpurun_out/cfg2s_$sw.log 2>&1 || { tail -20 gpurun_out/cfg2s_$sw.log; exit 1; }
  grep '"metric"' gpurun_out/cfg2s_$sw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg2 sw=$sw', r['value'], r['ms_per_step'])"
done
for sw in "" 1 "" 1; do
  LANGSTREAM_SWITCH_MS=$sw timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/rags_$sw.log 2>&1 || { tail -20 gpurun_out/rags_$sw.log; exit 1; }
  grep '"metric"' gpurun_out/rags_$sw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('rag sw=$sw', r['value'], r['p50_latency_s'], r['step_phases_rank0_s'])"
done
