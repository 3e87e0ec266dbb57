# r6: the round-end checks on the current tree: GPU suite, smoke, the headline bench with
# the driver's step counts, config 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6c}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$T.log 2>&1 || { tail -30 gpurun_out/bench20_$T.log; exit 1; }
tail -1 gpurun_out/bench20_$T.log | cut -c1-220
timeout -k 10 500 python -u bench.py --config chat --steps 3 --warmup 1 > gpurun_out/cfg3_$T.log 2>&1 || { tail -30 gpurun_out/cfg3_$T.log; exit 1; }
grep '"metric"' gpurun_out/cfg3_$T.log | cut -c1-200
