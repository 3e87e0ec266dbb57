# Decode attention at small-to-mid batch: single-split rows finished by the attention kernel
# (new) vs always merged (old), and the split target (TARGET_WG 1024 vs 512), one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4l}
cp abtmp/_hip_ops_new.so langstream_amd/ops/_hip_ops.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "decode_attn or decode_attention or paged_decode or graph or native_executor" > gpurun_out/attn_tests_$T.log 2>&1 || { tail -30 gpurun_out/attn_tests_$T.log; exit 1; }
tail -1 gpurun_out/attn_tests_$T.log
for r in 1 2; do
for v in old new; do
for tw in 1024 512; do
  cp abtmp/_hip_ops_$v.so langstream_amd/ops/_hip_ops.so
  echo "== $v target_wg $tw" >> gpurun_out/attn_split_$T.log
  LS_ATTN_TARGET_WG=$tw timeout -k 10 200 python -u tools/attn_bench.py --rope --ragged 0.3 --shapes 64x160,64x600,64x2048,32x600,128x600,16x2048 2>&1 | grep -v amdgpu | cut -c1-160 >> gpurun_out/attn_split_$T.log || exit 1
  LS_ATTN_TARGET_WG=$tw timeout -k 10 200 python -u tools/engine_bench.py --what llm --batch 64 --prompt 128 --gen 128 2>&1 | grep '"test"' | cut -c1-200 >> gpurun_out/attn_split_$T.log || exit 1
done; done; done
cat gpurun_out/attn_split_$T.log
