# LM head tile width A/B in the engine (LS_DGEMM_HEAD_BN 128 vs 256), B = 256 decode
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for bn in 128 256 128 256; do
  LS_DGEMM_HEAD_BN=$bn timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/headbn_$bn.log 2>&1 || { tail -20 gpurun_out/headbn_$bn.log; exit 1; }
  echo "bn=$bn $(grep -v amdgpu.ids gpurun_out/headbn_$bn.log | tail -1 | cut -c1-300)"
done
