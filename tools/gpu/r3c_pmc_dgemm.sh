# PMC passes over the decode gate_up GEMM (M = 256): L2 traffic and wave stall counters
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_dg
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_dg/p1 -o run --output-format csv -- python3 tools/dgemm_bench.py --only gate_up,down --rounds 1 --iters 5 > gpurun_out/pmc_dg/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_dg/p2 -o run --output-format csv -- python3 tools/dgemm_bench.py --only gate_up,down --rounds 1 --iters 5 > gpurun_out/pmc_dg/p2.log 2>&1 || exit $?
for p in p1 p2; do f=$(find gpurun_out/pmc_dg/$p -name "*counter_collection.csv" | head -1); python3 tools/pmc_summary.py "$f" dgemm_kernel; done > gpurun_out/pmc_dg/summary.txt
cat gpurun_out/pmc_dg/summary.txt
