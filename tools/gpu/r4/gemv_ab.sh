# GEMV prologue load-order A/B: old vs new _hip_ops.so on one box (gemv_bench + the
# prologue-norm GEMV tests), then batch-4 engine decode steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4g}
cp abtmp/_hip_ops_new.so langstream_amd/ops/_hip_ops.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv" > gpurun_out/gemv_tests_$T.log 2>&1 || { tail -30 gpurun_out/gemv_tests_$T.log; exit 1; }
tail -2 gpurun_out/gemv_tests_$T.log
for v in old new old new; do
  cp abtmp/_hip_ops_$v.so langstream_amd/ops/_hip_ops.so
  echo "== $v" >> gpurun_out/gemv_ab_$T.log
  timeout -k 10 200 python -u tools/gemv_bench.py --ts 1,4 >> gpurun_out/gemv_ab_$T.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/engine_bench.py --what llm --batch 4 --prompt 410 --gen 64 >> gpurun_out/gemv_ab_$T.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/gemv_ab_$T.log | cut -c1-260
