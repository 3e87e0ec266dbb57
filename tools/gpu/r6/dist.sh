# r6: one-shot all-reduce with uncached flags + bring-up self-check (RCCL world 1, multi-process on one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 180 --timeout-method thread -m gpu > gpurun_out/dist_r6.log 2>&1
rc=$?
tail -30 gpurun_out/dist_r6.log
exit $rc
