# round-4 call U: the co-running fp16 forward with no LDS-DMA conv at all
# (large tiles and the 256x256 split-K both off), then call T.
# Usage: bash tools/gpu_r4u.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
run() {  # name dtype mode dbg_set [env...]
  local name=$1 dt=$2 mode=$3 set=$4; shift 4
  env "$@" MDX_LIB_VARIANT=pk MDX_DEBUG_SHADOW=1 DBG_SET="$set" timeout -k 10 240 python3 -u tools/dbg_race.py $dt 30 $mode > $O/race_${name}_$T.log 2>&1 || { echo "race $name failed"; tail -5 $O/race_${name}_$T.log; return 1; }
  echo "$name: $(grep summary $O/race_${name}_$T.log)"
}
run nodma fp16 same "mdx_conv_set_large_tiles:0,mdx_conv_set_split256:0:18,mdx_conv_set_dma128:0:1536" && \
run a32b16nodma fp32 other "mdx_conv_set_large_tiles:0,mdx_conv_set_split256:0:18,mdx_conv_set_dma128:0:1536" DBG_OTHER_DT=fp16 && \
bash tools/gpu_r4t.sh $T
