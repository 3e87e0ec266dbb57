# r6: re-measure the prefill routing table (hipBLASLt vs gemm_pp_kernel per 256-row M
# bucket, median of 3 interleaved repeats), install it on this box, and A/B the headline
# bench: all hand-written (default) vs LS_PGEMM=route (plain projections on whichever
# measured faster), interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/route
timeout -k 10 400 python -u tools/pgemm_route_tune.py --out gpurun_out/route/pgemm_route_gfx950.csv > gpurun_out/route/tune.log 2>&1 || { tail -20 gpurun_out/route/tune.log; exit 1; }
cp gpurun_out/route/pgemm_route_gfx950.csv langstream_amd/ops/pgemm_route_gfx950.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/route/pgemm_route_gfx950.csv")))
for n in ("6144", "4096"):
    for k in ("4096", "14336"):
        sel = [r for r in rows if r["N"] == n and r["K"] == k]
        if sel:
            lib = sum(1 for r in sel if float(r["pp_us"]) >= 0.97 * float(r["lib_us"]))
            print(f"N={n} K={k}: {lib}/{len(sel)} buckets to the library;", " ".join(f'{r["M"]}:{r["lib_us"]}/{r["pp_us"]}' for r in sel[::8]))
PY
for r in 1 2; do
for mode in default route; do
  if [ $mode = route ]; then export LS_PGEMM=route; else unset LS_PGEMM; fi
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/route/bench20_${mode}_r$r.log 2>&1 || { tail -30 gpurun_out/route/bench20_${mode}_r$r.log; exit 1; }
  echo "$mode round $r"; tail -1 gpurun_out/route/bench20_${mode}_r$r.log | cut -c1-200
done
done
