# A/B of inpaint build variants (tools/build_variant.py): kbench at 1024 and 32
# frames per variant.  Usage (GPU box): bash tools/gpu_exp_inp.sh NAME...
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
test -f moseq2-detectron-extract_amd/libmdx.so || exit 5
for v in "$@"; do
  MDX_LIB_VARIANT=$v timeout -k 10 200 python3 -u tools/kbench.py --batch 1024 --reps 5 --only prep_inpaint > $O/exp_$v.log 2>&1 || exit 7
  MDX_LIB_VARIANT=$v timeout -k 10 200 python3 -u tools/kbench.py --batch 32 --only prep_inpaint >> $O/exp_$v.log 2>&1 || exit 7
done
echo rc=$?
