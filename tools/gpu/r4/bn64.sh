# BN = 64 decode GEMM tiles at M = 256 (qkv / o / down): correctness in the bench's own
# rel_err vs fp32, and time with the split-K reduction included.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4r}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dgemm_bench.py --ms 256,200 --only qkv,o,down --rounds 5 --iters 20 > gpurun_out/dgemm_bn64_$TAG.log 2>&1 || { tail -20 gpurun_out/dgemm_bn64_$TAG.log; exit 1; }
grep -v amdgpu gpurun_out/dgemm_bn64_$TAG.log | python3 -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: continue
    u=d['us']; e=d['rel_err']
    ks=[k for k in u if k.startswith('dgemm')]
    print(d['gemm'], d['M'], ' '.join(f'{k[6:]}={u[k]}' for k in ks), 'best', d['best'], 'maxerr', max(e.values()) if e else None)
"
