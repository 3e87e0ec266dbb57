# r6: kNN main pass with 4 waves x 64 queries (LS_KNN_NW=4: two MFMAs' worth more query
# fragments in registers per LDS row-fragment read) vs 8 waves x 32 (default): exactness
# tests under the variant, then Q = 256..2048 over 1M x 384 timed, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/knn
LS_KNN_NW=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k knn -x -q --timeout 120 --timeout-method thread > gpurun_out/knn/tests_nw4.log 2>&1
rc=$?; tail -2 gpurun_out/knn/tests_nw4.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for nw in 8 4; do
  LS_KNN_NW=$nw timeout -k 10 240 python -u tools/engine_bench.py --what knn --rows 1000000 --queries 256,1024,2048 > gpurun_out/knn/bench_nw${nw}_r$r.log 2>&1 || { tail -20 gpurun_out/knn/bench_nw${nw}_r$r.log; exit 1; }
  echo "NW=$nw round $r"; grep '"knn"' gpurun_out/knn/bench_nw${nw}_r$r.log
done
done
