# Full GPU check of the tree: pytest -m gpu, smoke(), the headline bench and its timed-window
# kernel timeline.  usage: bash tools/gpu/r3c_full.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r3c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
bash tools/gpu/r3_bench.sh $TAG
