# A/B: crawler agent in its own process (default) vs a thread of rank 0's runner, at the
# default 32 pages per step and at 256 (the crawl load rank 0 carries at 8 GPUs).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4p}
mkdir -p gpurun_out
for cfg in "0 32" "1 32" "0 32" "1 32" "0 256" "1 256"; do
set -- $cfg
LS_BENCH_CRAWLER_INPROC=$1 timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --docs $2 > gpurun_out/bench_cr$1_d$2_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_cr$1_d$2_$TAG.log; exit 1; }
echo "crawler_inproc=$1 docs=$2 $(grep '"metric"' gpurun_out/bench_cr$1_d$2_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_s"], d.get("ingest"))')"
done
