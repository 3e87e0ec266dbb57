# fused decode layer v2 (write-through slab publish, vectorised 1/rms loads): kernel tests,
# engine A/B, per-kernel stats of the fused engine run; then the W=8 kNN load and the
# config-2 stack profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "combine or silu_r or rms_prep or norm_deferred" > gpurun_out/fused_kernels2.log 2>&1
rc=$?; tail -n 3 gpurun_out/fused_kernels2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r4c.log 2>&1
rc=$?; tail -n 3 gpurun_out/gpu_tests_r4c.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  LS_DGEMM_FUSED=$f timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eng2_fused$f.log 2>&1 || { tail -20 gpurun_out/eng2_fused$f.log; exit 1; }
  echo "fused=$f $(grep -v amdgpu.ids gpurun_out/eng2_fused$f.log | tail -1 | cut -c1-260)"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o pf -- python3 tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/prof_fused.log 2>&1 || { tail -20 gpurun_out/prof_fused.log; exit 1; }
S=$(find gpurun_out/prof_fused -name '*kernel_stats.csv' | head -1)
python3 - "$S" << 'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:110]}')
PY
bash tools/gpu/r4/knn_w8_cfg2.sh
