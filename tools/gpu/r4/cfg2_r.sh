# config 2 replicas per GPU, interleaved on one box: R = 2, 3, 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4u}
mkdir -p gpurun_out
for R in 2 3 4 2 3 4; do
timeout -k 10 400 python -u bench.py --config embed --steps 5 --warmup 1 --batch 2048 --embed-replicas $R > gpurun_out/cfg2_${TAG}_R$R.log 2>&1 || { tail -30 gpurun_out/cfg2_${TAG}_R$R.log; exit 1; }
echo "R=$R $(grep '"metric"' gpurun_out/cfg2_${TAG}_R$R.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done
