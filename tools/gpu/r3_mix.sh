# headline bench (timeline) + configs 2/3/5 + decode attention in engine-like conditions
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r3_bench.sh r3b || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --shapes 256x410 --ragged 0.15 --pool-gb 100 > gpurun_out/attn_pool.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --shapes 256x410 --ragged 0.0 --pool-gb 100 >> gpurun_out/attn_pool.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --shapes 256x410 --ragged 0.15 --ring 4 >> gpurun_out/attn_pool.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --shapes 256x410 --ragged 0.0 --ring 4 >> gpurun_out/attn_pool.log 2>&1 || exit $?
cat gpurun_out/attn_pool.log | grep '"B"'
bash tools/gpu/r3_configs.sh
