# Single-LDS-stage k_conv (k_conv_sb, three / four workgroups per CU): tests,
# GEMM microbench A/B, bench A/B.  rc 1 does not stop the script; any other rc ends it.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp7_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp7_steps.txt; exit $rc; fi
}
run tE7.log timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q --timeout 120 --timeout-method thread -k "pointwise_instances or winograd"
run g32_sb0.log timeout -k 10 200 python3 -u tools/gemm32bench.py
run g32_sb1.log timeout -k 10 200 python3 -u tools/gemm32bench.py single_stage=1
B="--steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop"
run bE7_sb0.json timeout -k 10 300 python3 -u bench.py $B
run bE7_sb1.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_single_stage=1
run bE7_sb0b.json timeout -k 10 300 python3 -u bench.py $B
run bE7_sb1b.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_single_stage=1
echo done >> $O/exp7_steps.txt
