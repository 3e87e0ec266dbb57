# A/B: crawl site in its own process (default) vs in rank 0's interpreter.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4o}
mkdir -p gpurun_out
for v in 0 1 0 1; do
LS_BENCH_SITE_INPROC=$v timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_site${v}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_site${v}_$TAG.log; exit 1; }
echo "site_inproc=$v $(grep '"metric"' gpurun_out/bench_site${v}_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_s"])')"
done
