# round-4 call Q: bisect the fp16 forward's kernel mix that makes the
# packed-FP32 GN on the other stream differ (planner knobs are process-wide:
# they change the co-running forward's kernels; the GN kernels stay).
# Usage: bash tools/gpu_r4q.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
run() {  # name dbg_set
  MDX_LIB_VARIANT=pk MDX_DEBUG_SHADOW=1 DBG_SET="$2" timeout -k 10 240 python3 -u tools/dbg_race.py fp16 30 same > $O/race_${1}_$T.log 2>&1 || { echo "race $1 failed"; tail -5 $O/race_${1}_$T.log; return 1; }
  echo "$1 [$2]: $(grep summary $O/race_${1}_$T.log)"
}
run nostream "mdx_conv_set_stream1x1:0:65536" && \
run twostage "mdx_conv_set_single_stage:2" && \
run nolarge "mdx_conv_set_large_tiles:0" && \
run nosplit256 "mdx_conv_set_split256:0:18" && \
run nolarge_nostream "mdx_conv_set_large_tiles:0,mdx_conv_set_stream1x1:0:65536"
