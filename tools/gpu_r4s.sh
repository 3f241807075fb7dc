# round-4 call S: is the victim fp16-specific (an fp32 forward on A beside an
# fp16 forward on B), and does the co-running forward's ROIAlign variant matter.
# Usage: bash tools/gpu_r4s.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
run() {  # name dtype mode dbg_set [env...]
  local name=$1 dt=$2 mode=$3 set=$4; shift 4
  env "$@" MDX_LIB_VARIANT=pk MDX_DEBUG_SHADOW=1 DBG_SET="$set" timeout -k 10 240 python3 -u tools/dbg_race.py $dt 30 $mode > $O/race_${name}_$T.log 2>&1 || { echo "race $name failed"; tail -5 $O/race_${name}_$T.log; return 1; }
  echo "$name: $(grep summary $O/race_${name}_$T.log)"
}
run a32b16 fp32 other "" DBG_OTHER_DT=fp16 && \
run roi6 fp16 same "mdx_roi_align_set_mode:6" && \
run roiunsorted fp16 same "mdx_roi_align_set_sorted:0,mdx_roi_align_set_order:0"
