# PMC pass over the kNN search at Q=2048 (MFMA busy, wait buckets, LDS conflicts).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_knn_$TAG -o pm -- python3 tools/engine_bench.py --what knn --queries 2048 --iters 3 > gpurun_out/knn_pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/knn_pmc_$TAG.log; exit 1; }
F=$(find gpurun_out/pmc_knn_$TAG -name '*counter_collection.csv' | head -1)
python3 - "$F" << 'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "knn" not in k: continue
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %.4g" % (c, v))
PY
