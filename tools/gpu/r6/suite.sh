# r6: GPU suite + smoke on the current tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6h}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
