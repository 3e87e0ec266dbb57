# first-run slowness on a fresh box: byte-compile the package first, then config 2 twice
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ls langstream_amd/__pycache__ 2>/dev/null | head -3
t0=$(date +%s.%N); python -m compileall -q -j 8 langstream_amd bench.py > /dev/null; t1=$(date +%s.%N)
echo "compileall s: $(echo "$t1 - $t0" | bc)"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config embed --batch 2048 --steps 3 --warmup 1 > gpurun_out/cfg2c_$i.log 2>&1 || { tail -20 gpurun_out/cfg2c_$i.log; exit 1; }
  grep '"metric"' gpurun_out/cfg2c_$i.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg2 run $i', r['value'], r['ms_per_step'])"
done
