# Config 3: Llama-3-8B chat through the websocket gateway, 64 sessions; then the same run
# under rocprofv3 --kernel-trace --stats (library GEMM kernels must be absent).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4c3}
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --config chat --steps 3 --warmup 1 > gpurun_out/cfg3_$TAG.log 2>&1 || { tail -30 gpurun_out/cfg3_$TAG.log; exit 1; }
grep '"metric"' gpurun_out/cfg3_$TAG.log | cut -c1-400
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format rocpd -d gpurun_out/prof_cfg3_$TAG -o pc -- python3 bench.py --config chat --steps 2 --warmup 1 > gpurun_out/cfg3_prof_$TAG.log 2>&1 || { tail -30 gpurun_out/cfg3_prof_$TAG.log; exit 1; }
DB=$(find gpurun_out/prof_cfg3_$TAG -name '*.db' | head -1)
python3 tools/rocpd_stats.py $DB --top 25 > gpurun_out/cfg3_stats_$TAG.txt
head -14 gpurun_out/cfg3_stats_$TAG.txt | cut -c1-160
echo "library GEMM kernels: $(grep -c 'Cijk\|hipblaslt' gpurun_out/cfg3_stats_$TAG.txt || true)"
rm -f $DB
