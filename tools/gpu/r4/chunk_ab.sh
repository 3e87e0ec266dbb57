# Engine prefill chunk (max prefill tokens per step) A/B on the headline bench, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4z}
for r in 1 2; do
for c in 16384 32768 8192; do
  echo "== chunk $c" >> gpurun_out/chunk_ab_$T.log
  timeout -k 10 400 python -u bench.py --prefill-chunk $c 2>&1 | grep '"metric"' | cut -c1-260 >> gpurun_out/chunk_ab_$T.log || exit 1
done; done
cat gpurun_out/chunk_ab_$T.log
