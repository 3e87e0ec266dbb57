# Config 5's model at world 1: Llama-3-70B (140 GB bf16 on one GPU) chat through the gateway,
# then its kernel profile (library GEMM kernels must be absent).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4c5}
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --config chat --chat-model llama-3-70b --steps 2 --warmup 1 > gpurun_out/cfg5_$TAG.log 2>&1 || { tail -30 gpurun_out/cfg5_$TAG.log; exit 1; }
grep '"metric"' gpurun_out/cfg5_$TAG.log | cut -c1-500
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format rocpd -d gpurun_out/prof_cfg5_$TAG -o pc -- python3 bench.py --config chat --chat-model llama-3-70b --steps 1 --warmup 1 > gpurun_out/cfg5_prof_$TAG.log 2>&1 || { tail -30 gpurun_out/cfg5_prof_$TAG.log; exit 1; }
DB=$(find gpurun_out/prof_cfg5_$TAG -name '*.db' | head -1)
python3 tools/rocpd_stats.py $DB --top 25 > gpurun_out/cfg5_stats_$TAG.txt
head -14 gpurun_out/cfg5_stats_$TAG.txt | cut -c1-160
echo "library GEMM kernels: $(grep -c 'Cijk\|hipblaslt' gpurun_out/cfg5_stats_$TAG.txt || true)"
rm -f $DB
