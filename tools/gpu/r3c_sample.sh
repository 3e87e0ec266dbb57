# whole-process stack samples of the RAG bench (host pipeline: where the arrival spread goes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/stack_sampler.py --every-ms 10 --top 60 -- bench.py --steps 3 --warmup 1 > gpurun_out/sample_r3c.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/sample_r3c.log | grep '"metric"' | cut -c1-300; exit $rc
