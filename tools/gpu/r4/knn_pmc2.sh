# Second PMC pass over the kNN search at Q=2048: L2 hit/miss, LDS activity, issue stalls.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4h}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_${name}_$TAG -o pm -- python3 tools/engine_bench.py --what knn --queries 2048 --iters 3 > gpurun_out/knn_${name}_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_${name}_$TAG.log; return 1; }
  F=$(find gpurun_out/pmc_${name}_$TAG -name '*counter_collection.csv' | head -1)
  python3 - "$F" << 'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[r["Kernel_Name"][:70]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "knn" not in k: continue
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %.4g" % (c, v))
PY
}
run a TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run b TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE
