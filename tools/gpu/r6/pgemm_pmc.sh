# r6: PMC passes over the prefill ping-pong GEMM (and hipBLASLt on the same shapes, random
# operands) to prove its limiter: MFMA busy, LDS waits / conflicts, effective clock.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_pg
timeout -k 10 200 python3 -u tools/gemm_prefill_bench.py --ms 16384,4096 --only llama_gate_up,llama_down,llama_qkv,llama_o --ours --big > gpurun_out/pmc_pg/wall.log 2>&1 || { tail -20 gpurun_out/pmc_pg/wall.log; exit 1; }
cat gpurun_out/pmc_pg/wall.log
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_pg/p1 -o run -- python3 tools/gemm_prefill_bench.py --ms 16384 --only llama_gate_up,llama_down --ours --big > gpurun_out/pmc_pg/p1.log 2>&1 || { tail -20 gpurun_out/pmc_pg/p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_pg/p2 -o run -- python3 tools/gemm_prefill_bench.py --ms 16384 --only llama_gate_up,llama_down --ours --big > gpurun_out/pmc_pg/p2.log 2>&1 || { tail -20 gpurun_out/pmc_pg/p2.log; exit 1; }
for p in p1 p2; do f=$(find gpurun_out/pmc_pg/$p -name "*counter_collection.csv" | head -1); python3 tools/pmc_summary.py "$f"; done > gpurun_out/pmc_pg/summary.txt
cat gpurun_out/pmc_pg/summary.txt
