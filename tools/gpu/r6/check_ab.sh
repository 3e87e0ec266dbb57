# r6: GPU suite + smoke on the current tree, then the headline bench with the prefix KV
# cache on (default) and off (LS_PREFIX_CACHE=0) back to back on this box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6d}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
for v in 1 0; do
  LS_PREFIX_CACHE=$v timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20_prefix${v}_$T.log 2>&1 || { tail -30 gpurun_out/bench20_prefix${v}_$T.log; exit 1; }
  echo "LS_PREFIX_CACHE=$v"; tail -1 gpurun_out/bench20_prefix${v}_$T.log | cut -c1-240
done
