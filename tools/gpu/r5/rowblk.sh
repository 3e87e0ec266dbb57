# Decode GEMM at M = 256: row blocks without split-K (LS_DGEMM_ROWBLK) vs the split-K tiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5d}
timeout -k 10 300 python -u tools/dgemm_bench.py --ms 256,200 --only qkv,gate_up --rounds 5 > gpurun_out/rowblk_$T.log 2>&1 || { tail -30 gpurun_out/rowblk_$T.log; exit 1; }
cut -c1-900 gpurun_out/rowblk_$T.log
