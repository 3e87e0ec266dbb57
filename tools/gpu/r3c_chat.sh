# configs 3 and 5 (world 1) through the WebSocket chat gateway with this round's engine
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config chat --steps 3 --warmup 1 > gpurun_out/cfg3_r3c.log 2>&1 || { tail -20 gpurun_out/cfg3_r3c.log; exit 1; }
grep '"metric"' gpurun_out/cfg3_r3c.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg3', r['value'], r['ttft_p50_ms'], r['config'])"
timeout -k 10 600 python -u bench.py --config chat --chat-model llama-3-70b --steps 2 --warmup 1 > gpurun_out/cfg5_r3c.log 2>&1 || { tail -20 gpurun_out/cfg5_r3c.log; exit 1; }
grep '"metric"' gpurun_out/cfg5_r3c.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg5', r['value'], r['ttft_p50_ms'], r['config'])"
