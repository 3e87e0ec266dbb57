# Decode attention split target 512 (default) vs 256 at B = 8-32.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4aa}
for r in 1 2; do
for tw in 512 256; do
  echo "== target_wg $tw" >> gpurun_out/attn_split2_$T.log
  LS_ATTN_TARGET_WG=$tw timeout -k 10 200 python -u tools/attn_bench.py --rope --ragged 0.3 --shapes 32x300,32x600,32x2048,16x600,16x2048,8x2048 2>&1 | grep -v amdgpu | cut -c1-100 >> gpurun_out/attn_split2_$T.log || exit 1
  LS_ATTN_TARGET_WG=$tw timeout -k 10 200 python -u tools/engine_bench.py --what llm --batch 32 --prompt 410 --gen 128 2>&1 | grep '"test"' | cut -c1-200 >> gpurun_out/attn_split2_$T.log || exit 1
done; done
cat gpurun_out/attn_split2_$T.log
