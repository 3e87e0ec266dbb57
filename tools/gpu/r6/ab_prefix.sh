# r6: same-box A/B of the headline bench with the prefix KV cache on (default) and off
# (LS_PREFIX_CACHE=0), the driver's step counts, so the two sources of the round-5 gain
# stay separable.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abp
for v in 1 0; do
  LS_PREFIX_CACHE=$v timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/abp/bench20_prefix$v.log 2>&1 || { tail -30 gpurun_out/abp/bench20_prefix$v.log; exit 1; }
  echo "LS_PREFIX_CACHE=$v"; tail -1 gpurun_out/abp/bench20_prefix$v.log | cut -c1-200
done
