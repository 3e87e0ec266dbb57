# r6: two back-to-back headline bench runs (driver step counts) on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6j}
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20_${T}_$i.log 2>&1 || { tail -30 gpurun_out/bench20_${T}_$i.log; exit 1; }
  tail -1 gpurun_out/bench20_${T}_$i.log | cut -c1-200
done
