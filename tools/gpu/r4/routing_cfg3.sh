# Runner routing test at M = 5..700 rows vs fp32, then the B = 64 decode step (config 3
# shape) timed and under rocprofv3 --stats (library GEMM kernels must be absent).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4j}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q -k "routing_at_m_rows" --timeout 300 --timeout-method thread > gpurun_out/routing_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/routing_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 64 --prompt 410 --gen 128 > gpurun_out/eng_b64_$TAG.log 2>&1 || { tail -20 gpurun_out/eng_b64_$TAG.log; exit 1; }
grep -i "decode\|ms" gpurun_out/eng_b64_$TAG.log | tail -4
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd -d gpurun_out/prof_b64_$TAG -o pb -- python3 tools/engine_bench.py --what llm --batch 64 --prompt 410 --gen 128 > gpurun_out/prof_b64_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_b64_$TAG.log; exit 1; }
DB=$(find gpurun_out/prof_b64_$TAG -name '*.db' | head -1)
python3 tools/rocpd_stats.py $DB --top 25 > gpurun_out/b64_stats_$TAG.txt
head -16 gpurun_out/b64_stats_$TAG.txt
echo "library GEMM kernels:"; grep -c "Cijk\|hipblaslt" gpurun_out/b64_stats_$TAG.txt || true
rm -f $DB
