# r5: the driver's step counts (20 timed after 5 warmup), twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5x}
for i in 1 2; do
  timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20_${T}_$i.log 2>&1 || { tail -30 gpurun_out/bench20_${T}_$i.log; exit 1; }
  tail -1 gpurun_out/bench20_${T}_$i.log | cut -c1-250
done
