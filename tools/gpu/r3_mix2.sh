set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config embed > gpurun_out/cfg2_embed_b.log 2>&1 || { tail -20 gpurun_out/cfg2_embed_b.log; exit 1; }
grep '"metric"' gpurun_out/cfg2_embed_b.log | cut -c1-300
timeout -k 10 200 python -u tools/attn_bench.py --shapes 256x410 --ragged 0.15 --pool-gb 100 --rope > gpurun_out/attn_rope.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --shapes 256x410 --ragged 0.15 --pool-gb 100 --rope --interleave-gemm >> gpurun_out/attn_rope.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --shapes 256x410 --ragged 0.15 --pool-gb 100 --interleave-gemm >> gpurun_out/attn_rope.log 2>&1 || exit $?
grep '"B"' gpurun_out/attn_rope.log
bash tools/gpu/r3_pgemm.sh --ms 16384
