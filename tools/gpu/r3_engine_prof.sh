# per-kernel times of the B=256 decode loop (engine_bench) under rocprofv3 + an A/B of the engine step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/engprof -o ep -- python3 tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 64 > gpurun_out/engprof.log 2>&1 || { tail -20 gpurun_out/engprof.log; exit 1; }
DB=$(find gpurun_out/engprof -name '*.db' | head -1)
python3 tools/rocpd_stats.py $DB --grid --top 30 > gpurun_out/engine_kernel_stats.txt
head -32 gpurun_out/engine_kernel_stats.txt | cut -c1-200
rm -f $DB
for v in 0 1; do
  LS_QKV_ROPE=$v timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eb_qr$v.log 2>&1 || exit $?
  echo "LS_QKV_ROPE=$v $(tail -1 gpurun_out/eb_qr$v.log | cut -c1-260)"
done
