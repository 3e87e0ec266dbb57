# decode attention under engine-like conditions: sequential blocks, interleaved gate_up GEMM (power/cache), rocprof kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for args in "" "--seq-blocks" "--interleave-gemm" "--seq-blocks --interleave-gemm"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ae$i -o ae -- python3 tools/attn_bench.py --shapes 256x566 --uniform-lo 265 --sorted --ring 4 $args > gpurun_out/ae$i.log 2>&1 || { tail -5 gpurun_out/ae$i.log; exit 1; }
  grep '"B"' gpurun_out/ae$i.log | cut -c1-80
  f=$(find gpurun_out/ae$i -name '*kernel_stats.csv' | head -1)
  echo "[$args] $(grep decode_attn $f | head -1 | cut -d, -f1-8)"
done
