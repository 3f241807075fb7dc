# fp16 A/B of the fused conv3+shortcut GEMM (R50 B=32 and BASELINE config 5:
# R101 B=64), the extract loop (config 3) on the current tree.
# rc 1 does not stop the script; any other rc ends it.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp6_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp6_steps.txt; exit $rc; fi
}
B="--steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop"
run ext6.log env EXTRACT_AB=1 timeout -k 10 400 python3 -u tools/extract_bench.py 10000 1000 fp32
run bE6_f16.json timeout -k 10 300 python3 -u bench.py --dtype fp16 $B
run bE6_f16fuse.json timeout -k 10 300 python3 -u bench.py --dtype fp16 $B --set mdx_model_set_fuse_shortcut=2
run bE6_c5.json timeout -k 10 300 python3 -u bench.py --dtype fp16 --depth 101 --batch 64 $B
run bE6_c5fuse.json timeout -k 10 300 python3 -u bench.py --dtype fp16 --depth 101 --batch 64 $B --set mdx_model_set_fuse_shortcut=2
echo done >> $O/exp6_steps.txt
