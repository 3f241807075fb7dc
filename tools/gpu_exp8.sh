# Single-stage schedule for the general fp32 layers (k_conv_sbg, mode 2) and
# the Cin = 64 1x1 layers on k_conv_sb instead of the streaming kernel: tests,
# GEMM microbench and bench A/B.  rc 1 does not stop the script; any other rc ends it.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp8_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp8_steps.txt; exit $rc; fi
}
run tE8.log timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q --timeout 120 --timeout-method thread -k "single_stage_general or pointwise_instances"
run g32_s1.log timeout -k 10 200 python3 -u tools/gemm32bench.py
run g32_s2.log timeout -k 10 200 python3 -u tools/gemm32bench.py single_stage=2
B="--steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop"
run bE8_s1.json timeout -k 10 300 python3 -u bench.py $B
run bE8_s2.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_single_stage=2
run bE8_st0.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_stream1x1_f32=0
run bE8_s2st0.json timeout -k 10 300 python3 -u bench.py $B --set mdx_conv_set_single_stage=2 --set mdx_conv_set_stream1x1_f32=0
run bE8_s1b.json timeout -k 10 300 python3 -u bench.py $B
echo done >> $O/exp8_steps.txt
