# Llama-3-70B (world 1) batch 1-4 decode: before vs after the round-4 GEMV changes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4m}
for v in pregemv new new2; do
  cp abtmp/_hip_ops_$v.so langstream_amd/ops/_hip_ops.so
  for b in 1 3 4; do
    echo "== $v batch $b" >> gpurun_out/gemv70b_$T.log
    timeout -k 10 300 python -u tools/engine_bench.py --what llm --model llama-3-70b --batch $b --prompt 410 --gen 48 2>&1 | grep '"test"' | cut -c1-220 >> gpurun_out/gemv70b_$T.log || exit 1
  done
done
for v in new new2; do
  cp abtmp/_hip_ops_$v.so langstream_amd/ops/_hip_ops.so
  for b in 3 4; do
    echo "== 8b $v batch $b" >> gpurun_out/gemv70b_$T.log
    timeout -k 10 200 python -u tools/engine_bench.py --what llm --batch $b --prompt 410 --gen 64 2>&1 | grep '"test"' | cut -c1-220 >> gpurun_out/gemv70b_$T.log || exit 1
  done
done
cp abtmp/_hip_ops_new2.so langstream_amd/ops/_hip_ops.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_engine_gpu.py -k "gemv or batch1 or runner or native" > gpurun_out/gemv70b_tests_$T.log 2>&1 || { tail -30 gpurun_out/gemv70b_tests_$T.log; exit 1; }
tail -1 gpurun_out/gemv70b_tests_$T.log
cat gpurun_out/gemv70b_$T.log
