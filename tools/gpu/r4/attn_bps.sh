# Decode attention: fewest KV blocks per split 4 (default) vs 8 (short contexts single-split).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4ab}
for r in 1 2; do
for b in 4 8; do
  echo "== min_bps $b" >> gpurun_out/attn_bps_$T.log
  LS_ATTN_MIN_BPS=$b timeout -k 10 200 python -u tools/attn_bench.py --rope --ragged 0.3 --shapes 32x300,32x600,32x2048,16x600,16x2048,64x600,64x2048,256x448 2>&1 | grep -v amdgpu | cut -c1-100 >> gpurun_out/attn_bps_$T.log || exit 1
  LS_ATTN_MIN_BPS=$b timeout -k 10 200 python -u tools/engine_bench.py --what llm --batch 32 --prompt 410 --gen 128 2>&1 | grep '"test"' | cut -c1-200 >> gpurun_out/attn_bps_$T.log || exit 1
done; done
LS_ATTN_MIN_BPS=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "paged_decode or native_executor or graph" > gpurun_out/attn_bps_tests_$T.log 2>&1 || { tail -20 gpurun_out/attn_bps_tests_$T.log; exit 1; }
tail -1 gpurun_out/attn_bps_tests_$T.log
cat gpurun_out/attn_bps_$T.log
