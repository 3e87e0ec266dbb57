# BASELINE configs 2, 3 and 5 (world 1) through bench.py, logs to gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config embed > gpurun_out/cfg2_embed.log 2>&1 || { tail -20 gpurun_out/cfg2_embed.log; exit 1; }
grep '"metric"' gpurun_out/cfg2_embed.log | cut -c1-400
timeout -k 10 300 python -u bench.py --config chat > gpurun_out/cfg3_chat8b.log 2>&1 || { tail -20 gpurun_out/cfg3_chat8b.log; exit 1; }
grep '"metric"' gpurun_out/cfg3_chat8b.log | cut -c1-400
timeout -k 10 500 python -u bench.py --config chat --chat-model llama-3-70b --steps 2 --warmup 1 > gpurun_out/cfg5_chat70b_world1.log 2>&1 || { tail -20 gpurun_out/cfg5_chat70b_world1.log; exit 1; }
grep '"metric"' gpurun_out/cfg5_chat70b_world1.log | cut -c1-400
