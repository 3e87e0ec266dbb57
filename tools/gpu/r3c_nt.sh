# non-temporal weight / KV loads in the full RAG bench (timed-window timelines per setting)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm or wave_per_pair" -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_tests.log 2>&1
rc=$?; tail -2 gpurun_out/nt_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "LS_DGEMM_NTST=1" "LS_DGEMM_WNT=1" "LS_ATTN_NT=1" "LS_DGEMM_WNT=1 LS_ATTN_NT=1 LS_DGEMM_NTST=1"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/tl_$tag -o tl -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_$tag.log 2>&1 || exit $?
  DB=$(find gpurun_out/tl_$tag -name '*.db' | head -1)
  MS=$(grep '"metric"' gpurun_out/bench_$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*3/1000)')
  python3 tools/timeline_window.py $DB --window-s $MS --top 12 > gpurun_out/timeline_$tag.txt
  rm -f $DB
  echo "== $cfg $(grep '"metric"' gpurun_out/bench_$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  sed -n 15,24p gpurun_out/timeline_$tag.txt | cut -c1-90
done
