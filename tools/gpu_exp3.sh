# Session-2 experiments, part 2: the fused conv3+shortcut tests and forward
# parity, the ROIAlign LDS-window mode, the config-3 extract loop, per-layer
# conv dumps with and without the fusion, and which file's packed-FP32 build
# makes the fp16 pipelined loop nondeterministic (pkm: model_ops.hip packed,
# pkc: conv.hip + inpaint.hip packed; default build: none of the three).
# rc 1 (a failed check) does not stop the script; any other rc ends it.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() {  # run LOG CMD...
  local log=$1; shift
  "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/exp3_steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $log (rc=$rc)" >> $O/exp3_steps.txt; exit $rc; fi
}
run tE3a.log timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q --timeout 120 --timeout-method thread -k "dual or fused_shortcut or winograd"
run det16.log timeout -k 10 300 python3 -u tools/determinism.py fp16 150
run det16pkm.log env MDX_LIB_VARIANT=pkm timeout -k 10 300 python3 -u tools/determinism.py fp16 150
run det16pkc.log env MDX_LIB_VARIANT=pkc timeout -k 10 300 python3 -u tools/determinism.py fp16 150
run det32pkc.log env MDX_LIB_VARIANT=pkc timeout -k 10 300 python3 -u tools/determinism.py fp32 150
run roi32.log timeout -k 10 200 python3 -u tools/roibench.py fp32
run bE3_dump0.json timeout -k 10 300 python3 -u bench.py --steps 20 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop --dump-convs $O/convs_fuse0.json
run bE3_dump1.json timeout -k 10 300 python3 -u bench.py --steps 20 --no-secondary --no-cpu-baseline --no-roofline --no-extract-loop --set mdx_model_set_fuse_shortcut=1 --dump-convs $O/convs_fuse1.json
run ext3.log timeout -k 10 400 python3 -u tools/extract_bench.py 10000 1000 fp32
echo done >> $O/exp3_steps.txt
