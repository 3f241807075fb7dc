# fp16: the register-staged single-stage kernel (mdx_conv_set_single_stage(3))
# with and without the LDS-DMA big-layer kernels, R50 B=32 and config 5.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp10_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp10_steps.txt; exit $rc; fi
}
B="--dtype fp16 --steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop"
run b10_base.json timeout -k 10 300 python3 -u bench.py $B
run b10_sb3.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_single_stage=3
run b10_sb3_nolarge.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_single_stage=3 --set mdx_conv_set_large_tiles=0
run b10_nolarge.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_large_tiles=0
run b10_c5_base.json timeout -k 10 300 python3 -u bench.py $B --depth 101 --batch 64
run b10_c5_sb3.json timeout -k 10 300 python3 -u bench.py $B --depth 101 --batch 64 --set mdx_conv_set_single_stage=3
run b10_c5_sb3_nolarge.json timeout -k 10 300 python3 -u bench.py $B --depth 101 --batch 64 --set mdx_conv_set_single_stage=3 --set mdx_conv_set_large_tiles=0
echo done >> $O/exp10_steps.txt
