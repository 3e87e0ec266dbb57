# r5: decode attention cache policy in the RAG bench, same box: LS_ATTN_NT=2 (first block
# cached, default) vs 1 (all nt), kernel timelines of the timed window.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for nt in 2 1; do
  LS_ATTN_NT=$nt timeout -k 10 500 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/tlnt$nt -o tl -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/bench_nt$nt.log 2>&1 || { tail -20 gpurun_out/bench_nt$nt.log; exit 1; }
  DB=$(find gpurun_out/tlnt$nt -name '*.db' | head -1)
  MS=$(grep '"metric"' gpurun_out/bench_nt$nt.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*3/1000)')
  python3 tools/timeline_window.py $DB --window-s $MS --top 12 > gpurun_out/timeline_nt$nt.txt
  echo "== NT=$nt $(grep -o '"value": [0-9.]*' gpurun_out/bench_nt$nt.log | head -1)"
  grep -E "decode_attn|window" gpurun_out/timeline_nt$nt.txt | head -4
  rm -f $DB
done
