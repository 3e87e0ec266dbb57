# r6: decode-shape GEMMs at M = 256 / 128 with cold weights: the decode kernels vs the
# prefill 256x256 ping-pong kernel (ops.gemm_prefill) on the same shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dpp
timeout -k 10 400 python3 -u tools/dgemm_bench.py --ms 256,128 --rounds 3 --iters 20 > gpurun_out/dpp/dgemm_pp.log 2>&1 || { tail -30 gpurun_out/dpp/dgemm_pp.log; exit 1; }
grep '^{' gpurun_out/dpp/dgemm_pp.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); u=r['us']
    keep={k:v for k,v in u.items() if k.startswith(('pgemm','dgemm_s','dgemm_bn128_s0','dgemm_bn128_s4','dgemm_bn128_s8','hipblas'))}
    print(r['gemm'], r['M'], 'best', r['best'], u[r['best']], keep)
"
