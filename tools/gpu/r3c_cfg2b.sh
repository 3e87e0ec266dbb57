# config 2 (compute-ai-embeddings on Kafka records) with the native JSON encoder + host stack samples
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 256 2048; do
  timeout -k 10 300 python -u bench.py --config embed --batch $b --steps 3 --warmup 1 > gpurun_out/cfg2j_b$b.log 2>&1 || { tail -20 gpurun_out/cfg2j_b$b.log; exit 1; }
  grep '"metric"' gpurun_out/cfg2j_b$b.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print($b, r['value'], r['ms_per_step'])"
done
timeout -k 10 300 python -u tools/stack_sampler.py --every-ms 5 --top 50 -- bench.py --config embed --batch 2048 --steps 3 --warmup 1 > gpurun_out/cfg2j_prof.log 2> gpurun_out/cfg2j_prof.err
