# The prefill GEMM kernel at decode-sized M (256, 512) vs the decode GEMM path (warm weights).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4n}
timeout -k 10 300 python -u tools/pgemm_ab.py --ms 256,512 --variants 1,3,4 --rounds 3 2>&1 | grep gemm > gpurun_out/pp256_$T.log || exit 1
timeout -k 10 300 python -u tools/dgemm_bench.py --ms 256 --only qkv,gate_up,down --rounds 3 --iters 20 2>&1 | grep gemm | cut -c1-400 >> gpurun_out/pp256_$T.log || exit 1
cat gpurun_out/pp256_$T.log | cut -c1-400
