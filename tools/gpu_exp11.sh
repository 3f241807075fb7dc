# Extract loop: cross-chunk pipeline A/B, each order in its own process (the
# first session of a process is the bench secondary's case); narrow-tile K
# threshold A/B for the fp32 loop.  rc 1 does not stop the script.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp11_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp11_steps.txt; exit $rc; fi
}
run ext11a.log env EXTRACT_AB=1 EXTRACT_AB_ORDER=1,0,1,0 timeout -k 10 500 python3 -u tools/extract_bench.py 10000 1000 fp32
run ext11b.log env EXTRACT_AB=1 EXTRACT_AB_ORDER=0,1,0,1 timeout -k 10 500 python3 -u tools/extract_bench.py 10000 1000 fp32
B="--steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop"
run b11_nk128.json timeout -k 10 300 python3 -u bench.py $B
run b11_nk64.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_narrow_kmax=64
run b11_nk256.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_narrow_kmax=256
echo done >> $O/exp11_steps.txt
