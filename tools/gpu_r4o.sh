# round-4 call O: which co-running work makes the packed-FP32 GN differ:
# a second handle (fp16 / fp32) on stream B, and the lone conv / GN
# backgrounds long enough (DBG_BG=40) to cover the whole forward on A.
# Usage: bash tools/gpu_r4o.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
run() {  # name mode [env...]
  local name=$1 mode=$2; shift 2
  env "$@" MDX_LIB_VARIANT=pk MDX_DEBUG_SHADOW=1 timeout -k 10 240 python3 -u tools/dbg_race.py fp16 30 $mode > $O/race_${name}_$T.log 2>&1 || { echo "race $name failed"; tail -5 $O/race_${name}_$T.log; return 1; }
  echo "$name: $(grep summary $O/race_${name}_$T.log)"
}
run other16 other DBG_OTHER_DT=fp16 && run other32 other DBG_OTHER_DT=fp32 && \
run conv40 conv DBG_BG=40 && run gn40 gn DBG_BG=40 && run same same
