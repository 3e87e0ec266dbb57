# 512-thread split-K add+RMSNorm A/B; attention after an interleaved copy vs GEMM (cache/TLB vs clock)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm or skinny" -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests_norm.log 2>&1
rc=$?; tail -2 gpurun_out/dg_tests_norm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dgemm_bench.py --only o,down --rounds 7 --env-ab LS_NORM_NT512 > gpurun_out/dg_norm.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/dg_norm.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['gemm'], {k:v for k,v in r['us'].items() if 'bn256' not in k})"
i=5
for args in "--interleave-copy" "--interleave-gemm"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace -d gpurun_out/ae$i -o ae -- python3 tools/attn_bench.py --shapes 256x566 --uniform-lo 265 --sorted --ring 4 $args > gpurun_out/ae$i.log 2>&1 || { tail -5 gpurun_out/ae$i.log; exit 1; }
  echo "[$args] $(python3 tools/rocpd_stats.py $(find gpurun_out/ae$i -name '*.db' | head -1) --top 3 | grep decode_attn | cut -d, -f1-6)"
done
