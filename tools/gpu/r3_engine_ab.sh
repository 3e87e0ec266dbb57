set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 1; do
  LS_DGEMM=$v timeout -k 10 300 python -u tools/engine_bench.py --what llm --batch 256 --prompt 410 --gen 128 > gpurun_out/eb_dg$v.log 2>&1 || exit $?
  echo "LS_DGEMM=$v $(tail -1 gpurun_out/eb_dg$v.log | cut -c1-330)"
done
