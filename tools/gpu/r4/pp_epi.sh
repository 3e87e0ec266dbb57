# Prefill GEMM epilogue A/B: ping-pong kernel with scattered 2-B stores (v1) vs LDS-staged
# 16-B row stores (v3) vs no stores (v4, timing ablation); hipBLASLt for reference; then
# the tile-group size (LS_PGEMM_GROUP) on the plain shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pgemm_ab.py --ms 4096,16384 --variants 1,3,4 --rounds 5 > gpurun_out/pp_epi.log 2>&1 || { tail -20 gpurun_out/pp_epi.log; exit 1; }
grep -v amdgpu gpurun_out/pp_epi.log
for g in 4 16; do
  LS_PGEMM_GROUP=$g timeout -k 10 200 python -u tools/pgemm_ab.py --ms 16384 --variants 1,3 --only qkv,o,down --rounds 3 > gpurun_out/pp_group$g.log 2>&1 || { tail -20 gpurun_out/pp_group$g.log; exit 1; }
  echo "group=$g"; grep -v amdgpu gpurun_out/pp_group$g.log
done
