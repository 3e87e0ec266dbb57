# kNN main pass ablations at Q = 1024 / 2048 (timing only): 0 full, 1 no sync, 2 no sync + no DMA, 3 no MFMA.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4w}
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in 0 1 2 3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd -d gpurun_out/prof_kabl${a}_$TAG -o pk -- python3 tools/engine_bench.py --what knn --queries 2048 --iters 10 --knn-ablate $a > gpurun_out/knn_abl${a}_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_abl${a}_$TAG.log; exit 1; }
DB=$(find gpurun_out/prof_kabl${a}_$TAG -name '*.db' | head -1)
echo "abl=$a $(python3 tools/rocpd_stats.py $DB --top 3 | grep 'q256_kernel<384, 1' | cut -d, -f1-4)"
rm -f $DB
done
