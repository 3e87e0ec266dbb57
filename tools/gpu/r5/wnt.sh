# r5: decode step at B = 256 (engine_bench) with the weight-load cache policy
# LS_DGEMM_WNT = 1 (all nt), 2 (nt past 64 MB: gate_up / down), 0 (none), twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
for v in 1 2 0; do
  LS_DGEMM_WNT=$v timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 --iters 3 > gpurun_out/wnt${v}_$r.log 2>&1 || { tail -20 gpurun_out/wnt${v}_$r.log; exit 1; }
  echo "WNT=$v run $r: $(grep -i -E 'decode' gpurun_out/wnt${v}_$r.log | tail -2 | cut -c1-250)"
done
done
