# Box pooler A/B: the ROIAlign GPU tests on the default library, then kernel
# traces of serial bench steps with the default library and with a variant
# (MDX_LIB_VARIANT=$2, built by tools/build_variant.py), and the per-launch
# ROIAlign durations of both (tools/roi_trace.py).
# Usage (GPU box): bash tools/gpu_roi_ab.sh TAG VARIANT [VARIANT2]
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=${1:-x}
V=${2:-roiold}
test -f moseq2-detectron-extract_amd/libmdx.so || exit 5
V2=$3
test -f moseq2-detectron-extract_amd/libmdx_$V.so || exit 6
B="--steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-roofline --no-overlap"
timeout -k 10 300 python3 -u -m pytest tests/test_model_gpu.py -x -q -k "roi_align" --timeout 120 --timeout-method thread > $O/roi_t$T.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/roi_new$T -o t --output-format csv -- python3 bench.py $B > $O/roi_new$T.log 2>&1 && \
MDX_LIB_VARIANT=$V timeout -k 10 200 rocprofv3 --kernel-trace -d $O/roi_old$T -o t --output-format csv -- python3 bench.py $B > $O/roi_old$T.log 2>&1 && \
if [ -n "$V2" ]; then MDX_LIB_VARIANT=$V2 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/roi_v2$T -o t --output-format csv -- python3 bench.py $B > $O/roi_v2$T.log 2>&1; fi && \
python3 tools/roi_trace.py $(find $O/roi_new$T $O/roi_old$T $O/roi_v2$T -name '*kernel_trace.csv' 2>/dev/null) > $O/roi_ab$T.txt 2>&1
echo "rc=$?" >> $O/roi_t$T.log
