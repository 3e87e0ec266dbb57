# config 2 with native JSON + native Kafka records; per-thread cProfile of one run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 256 2048; do
  timeout -k 10 300 python -u bench.py --config embed --batch $b --steps 3 --warmup 1 > gpurun_out/cfg2k_b$b.log 2>&1 || { tail -20 gpurun_out/cfg2k_b$b.log; exit 1; }
  grep '"metric"' gpurun_out/cfg2k_b$b.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print($b, r['value'], r['ms_per_step'])"
done
timeout -k 10 300 python -u tools/thread_cprofile.py --top 70 -- bench.py --config embed --batch 4096 --steps 4 --warmup 1 > gpurun_out/cfg2k_prof.log 2> gpurun_out/cfg2k_prof.err
