# r5: whole GPU suite + smoke + headline bench on the current tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r5t}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
timeout -k 10 500 python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_$T.log 2>&1 || { tail -30 gpurun_out/bench_$T.log; exit 1; }
tail -1 gpurun_out/bench_$T.log | cut -c1-250
