# Pointwise (per-row precomputed address) k_conv instances: conv tests, GEMM
# microbench A/B, bench A/B.  rc 1 does not stop the script; any other rc ends it.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp4_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp4_steps.txt; exit $rc; fi
}
run tE4.log timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_predictor_parity.py -q --timeout 200 --timeout-method thread -k "conv or winograd or dual or fused or backbone or predictor or forward_fp32"
run g32_pw1.log timeout -k 10 200 python3 -u tools/gemm32bench.py
run g32_pw0.log timeout -k 10 200 python3 -u tools/gemm32bench.py pointwise=0
run bE4_pw1.json timeout -k 10 300 python3 -u bench.py --steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop
run bE4_pw0.json timeout -k 10 300 python3 -u bench.py --steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop --set mdx_conv_set_pointwise=0
run bE4_pw1b.json timeout -k 10 300 python3 -u bench.py --steps 60 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop
echo done >> $O/exp4_steps.txt
