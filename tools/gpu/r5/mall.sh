# r5: decode GEMMs at M = 256 with the weights cold (rotated past the Infinity Cache) vs
# cache-resident (one copy), each with non-temporal W loads on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dgemm_bench.py --ms 256 --only qkv,o,down,gate_up --rounds 5 --iters 20 --env-ab LS_DGEMM_WNT > gpurun_out/dgemm_cold_r5q.log 2>&1 || { tail -20 gpurun_out/dgemm_cold_r5q.log; exit 1; }
timeout -k 10 300 python -u tools/dgemm_bench.py --ms 256 --only qkv,o,down,gate_up --rounds 5 --iters 20 --ring 1 --env-ab LS_DGEMM_WNT > gpurun_out/dgemm_hot_r5q.log 2>&1 || { tail -20 gpurun_out/dgemm_hot_r5q.log; exit 1; }
