# Box head FCs on k_conv_sb (LDS-DMA 256x256 kernel off) vs the default.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp9_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp9_steps.txt; exit $rc; fi
}
B="--steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop"
run bE9_d2.json timeout -k 10 300 python3 -u bench.py $B
run bE9_d0.json timeout -k 10 300 python3 -u bench.py $B --dma-f32 0
run bE9_d0dump.json timeout -k 10 300 python3 -u bench.py --steps 10 --no-secondary --no-cpu-baseline --no-extract-loop --dma-f32 0 --dump-convs $O/convs_d0.json
echo done >> $O/exp9_steps.txt
