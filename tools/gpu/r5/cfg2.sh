# r5: config 2 with ONE agent process (R = 1), twice, and with the default 3 replicas.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5j}
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --config embed --steps 5 --warmup 1 --batch 2048 --embed-replicas 1 > gpurun_out/cfg2_${T}_R1_$i.log 2>&1 || { tail -30 gpurun_out/cfg2_${T}_R1_$i.log; exit 1; }
  tail -1 gpurun_out/cfg2_${T}_R1_$i.log | cut -c1-200
done
timeout -k 10 400 python -u bench.py --config embed --steps 5 --warmup 1 --batch 2048 > gpurun_out/cfg2_${T}_R3.log 2>&1 || { tail -30 gpurun_out/cfg2_${T}_R3.log; exit 1; }
tail -1 gpurun_out/cfg2_${T}_R3.log | cut -c1-200
LS_STAGE_TRACE=1 timeout -k 10 500 python -u bench.py --steps 3 --warmup 2 > gpurun_out/bench_stage_${T}.log 2>&1 || { tail -30 gpurun_out/bench_stage_${T}.log; exit 1; }
tail -1 gpurun_out/bench_stage_${T}.log | cut -c1-200
