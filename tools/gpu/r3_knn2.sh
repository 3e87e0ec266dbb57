set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "knn" > gpurun_out/knn_tests2.log 2>&1 || { tail -30 gpurun_out/knn_tests2.log; exit 1; }
tail -1 gpurun_out/knn_tests2.log
timeout -k 10 200 python -u tools/engine_bench.py --what knn --rows 1000000 --queries 64,256,512,1024,2048 > gpurun_out/knn_bench2.log 2>&1 || { tail -20 gpurun_out/knn_bench2.log; exit 1; }
grep knn gpurun_out/knn_bench2.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/knnprof2 -o kp -- python3 tools/engine_bench.py --what knn --rows 1000000 --queries 1024,2048 > gpurun_out/knnprof2.log 2>&1 || { tail -20 gpurun_out/knnprof2.log; exit 1; }
LS_BENCH_FORCE_DIST=1 LS_KNN_REPLICATE=8 LS_KNN_PROFILE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --steps 3 --warmup 1 > gpurun_out/bench_forcedist_rep8.log 2>&1 || { tail -20 gpurun_out/bench_forcedist_rep8.log; exit 1; }
grep -o '"knn_rounds_per_rank.*' gpurun_out/bench_forcedist_rep8.log | cut -c1-600
grep '"metric"' gpurun_out/bench_forcedist_rep8.log | cut -c1-200
