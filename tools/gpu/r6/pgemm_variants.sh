# r6: prefill GEMM variants A/B (LS_PGEMM_KERNEL 1 = ping-pong default, 2 = persistent,
# 3 = ping-pong with the LDS-staged full-line epilogue), two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pgv
for r in 1 2; do
for v in 1 2 3; do
  LS_PGEMM_KERNEL=$v timeout -k 10 240 python3 -u tools/gemm_prefill_bench.py --ms 16384,12288,4096 --only llama_gate_up,llama_down,llama_qkv,llama_o --ours --big > gpurun_out/pgv/v${v}_r$r.log 2>&1 || { tail -20 gpurun_out/pgv/v${v}_r$r.log; exit 1; }
  echo "== v$v round $r"; grep -o '"M": [0-9]*, "gemm": "[a-z_]*".*"ours_us": [0-9.]*' gpurun_out/pgv/v${v}_r$r.log | sed 's/"N".*"ours_us"/ours_us/'
done
done
