# r5: per-kernel times of the B = 256 decode step, default layer vs the norm-deferred
# fused layer (LS_DGEMM_FUSED=1), from rocprofv3 kernel traces of engine_bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  LS_DGEMM_FUSED=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/prof_fused$v -o pc -- python3 tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 64 --iters 2 > gpurun_out/fused_prof$v.log 2>&1 || { tail -20 gpurun_out/fused_prof$v.log; exit 1; }
  grep -o '"ms_per_decode_step": [0-9.]*' gpurun_out/fused_prof$v.log | tail -1
  DB=$(find gpurun_out/prof_fused$v -name '*.db' | head -1)
  python3 tools/rocpd_stats.py $DB --top 22 > gpurun_out/fused_stats$v.txt
  rm -f $DB
done
