# paired-row decode attention A/B (LS_ATTN_PAIR, engine-ordered rows) + 2-rank native TP test
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_attention or decode_attn" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
for pr in 0 1; do
  for args in "--shapes 256x410" "--shapes 256x566 --uniform-lo 265 --sorted" "--shapes 256x566 --uniform-lo 265" "--shapes 256x1024 --uniform-lo 512 --sorted" "--shapes 128x410"; do
    LS_ATTN_PAIR=$pr timeout -k 10 120 python -u tools/attn_bench.py $args --ring 4 --check-all 2>&1 | grep '"B"' || exit 1
  done
done
timeout -k 10 240 python -u -m pytest tests/test_engine_gpu.py -k "tp2_two_ranks" -x -v --timeout 200 --timeout-method thread > gpurun_out/tp2_tests.log 2>&1
rc=$?; tail -4 gpurun_out/tp2_tests.log; [ $rc -eq 0 ] || exit $rc
