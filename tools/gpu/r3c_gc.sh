# GC young-generation threshold A/B on one box (3 timed steps each, alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for g in 50000 400000 50000 400000; do
  LANGSTREAM_GC_GEN0=$g timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_gc$g.log 2>&1 || exit $?
  grep '"metric"' gpurun_out/bench_gc$g.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print($g, r['value'], r['gc_rank0'])"
done
