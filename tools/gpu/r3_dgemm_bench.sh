set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/dgemm_bench.py "$@" > gpurun_out/dg_bench.log 2>&1 || exit $?
cat gpurun_out/dg_bench.log
