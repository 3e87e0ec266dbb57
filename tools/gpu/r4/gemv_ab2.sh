# gate_up prologue threshold (LS_GEMV_PRO_MAX_T) at batch 1-4 decode, interleaved on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4h}
cp abtmp/_hip_ops_new.so langstream_amd/ops/_hip_ops.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "gemv or batch1 or runner" > gpurun_out/gemv_tests_$T.log 2>&1 || { tail -30 gpurun_out/gemv_tests_$T.log; exit 1; }
tail -2 gpurun_out/gemv_tests_$T.log
timeout -k 10 200 python -u tools/gemv_bench.py --ts 2,3 >> gpurun_out/gemv_ab_$T.log 2>&1 || exit 1
for r in 1 2; do
for b in 1 2 3 4; do
for p in 4 2; do
  echo "== batch $b pro_max_t $p" >> gpurun_out/gemv_ab_$T.log
  LS_GEMV_PRO_MAX_T=$p timeout -k 10 200 python -u tools/engine_bench.py --what llm --batch $b --prompt 410 --gen 64 2>&1 | grep '"test"' | cut -c1-200 >> gpurun_out/gemv_ab_$T.log || exit 1
done; done; done
grep -v amdgpu.ids gpurun_out/gemv_ab_$T.log | cut -c1-260
