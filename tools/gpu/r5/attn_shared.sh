# r5: decode attention at B = 256 (contexts 270..550, the bench's), cold caches (ring of
# pools past the Infinity Cache), with 0 or 1 shared first block, nt policies 0 / 1 / 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/attn_shared_r5ab.log
: > $OUT
for sf in 0 1; do for nt in 1 2 0; do
  LS_ATTN_NT=$nt timeout -k 10 120 python -u tools/attn_bench.py --shapes 256x550 --uniform-lo 270 --ring 4 --shared-first $sf >> $OUT 2>&1 || { tail -20 $OUT; exit 1; }
done; done
grep '^{' $OUT | cut -c1-200
