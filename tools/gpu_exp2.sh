# Round-3 session-2 experiments: the fused conv3+shortcut GEMM (tests, bench
# A/B), the fp32 GEMM kernel A/B (k_conv vs k_conv_m32 vs persistent
# k_gemm_m32p), vectorised Winograd transforms, the LDS-window ROIAlign, and
# the packed-FP32 determinism A/B.  A step that fails normally (rc 1) does not
# stop the script; a fault, abort, signal or time limit (any other rc) ends it.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp2_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp2_steps.txt; exit $rc; fi
}
run tE2a.log timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q --timeout 120 --timeout-method thread -k "dual or fused_shortcut or backbone"
run bE2_base.json timeout -k 10 300 python3 -u bench.py --steps 40 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop
run bE2_fuse.json timeout -k 10 300 python3 -u bench.py --steps 40 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop --set mdx_model_set_fuse_shortcut=1
run g32_base.log timeout -k 10 200 python3 -u tools/gemm32bench.py
run g32_m32.log timeout -k 10 200 python3 -u tools/gemm32bench.py f32_mfma32=1
run g32_m32p.log timeout -k 10 200 python3 -u tools/gemm32bench.py f32_mfma32=2
run g32_m32pv.log timeout -k 10 200 python3 -u tools/gemm32bench.py f32_mfma32=2 wino_vec=1
run g32_vec.log timeout -k 10 200 python3 -u tools/gemm32bench.py wino_vec=1
run roi32.log timeout -k 10 200 python3 -u tools/roibench.py fp32
run tE2b.log timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "m32 or inpaint or winograd or roi_align"
run det32pk.log env MDX_LIB_VARIANT=pk timeout -k 10 300 python3 -u tools/determinism.py fp32 150
run det16pk.log env MDX_LIB_VARIANT=pk timeout -k 10 300 python3 -u tools/determinism.py fp16 150
run bE2_pk.json env MDX_LIB_VARIANT=pk timeout -k 10 300 python3 -u bench.py --steps 40 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop
echo done >> $O/exp2_steps.txt
