# config 2 pipeline: whole-process stack samples on the GPU box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stack_sampler.py --every-ms 2 --top 40 -- bench.py --config embed --batch 4096 --steps 3 --warmup 1 > gpurun_out/cfg2_prof.log 2> gpurun_out/cfg2_prof.err || { tail -20 gpurun_out/cfg2_prof.err; exit 1; }
grep '"metric"' gpurun_out/cfg2_prof.log | cut -c1-200
head -60 gpurun_out/cfg2_prof.err
