# decode-attention A/B on the GPU box: kernel tests, then tools/attn_bench.py per variant
set -e
cd /root/repo
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "decode_attention" > gpurun_out/attn_tests.log 2>&1
variants=("$@")
[ ${#variants[@]} -eq 0 ] && variants=(4:0 4:1 1:0 1:1)
for v in "${variants[@]}"; do
  w=${v%%:*}; p=${v##*:}
  echo "== WPP=$w PIPE=$p" >> gpurun_out/attn_ab.log
  LS_ATTN_WPP=$w LS_ATTN_PIPE=$p timeout -k 10 300 python -u tools/attn_bench.py --check-all >> gpurun_out/attn_ab.log 2>&1
done
