# r5: config 2, one agent process, longer window (20 timed steps after 3 warmup), twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5k}
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --config embed --steps 20 --warmup 3 --batch 2048 --embed-replicas 1 > gpurun_out/cfg2_long_${T}_$i.log 2>&1 || { tail -30 gpurun_out/cfg2_long_${T}_$i.log; exit 1; }
  tail -1 gpurun_out/cfg2_long_${T}_$i.log | cut -c1-200
done
