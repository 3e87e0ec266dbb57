# Per-kernel breakdown of the kNN search at Q=1024/2048 over 1M x 384.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4e}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd -d gpurun_out/prof_knn_$TAG -o pk -- python3 tools/engine_bench.py --what knn --queries 2048 --iters 20 > gpurun_out/knn_prof_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_prof_$TAG.log; exit 1; }
DB=$(find gpurun_out/prof_knn_$TAG -name '*.db' | head -1)
python3 tools/rocpd_stats.py $DB --grid --top 20 > gpurun_out/knn_prof_stats_$TAG.txt
cat gpurun_out/knn_prof_stats_$TAG.txt
rm -f $DB
