# round-4 call Z: trunk or heads -- the packed GN on A beside a second handle
# on B in the mixed configuration (fp32 trunk / RPN / box head, fp16 mask and
# keypoint heads), both A dtypes.  Usage: bash tools/gpu_r4z.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
run() {  # name dtype mode dbg_set [env...]
  local name=$1 dt=$2 mode=$3 set=$4; shift 4
  env "$@" MDX_LIB_VARIANT=pk MDX_DEBUG_SHADOW=1 DBG_SET="$set" timeout -k 10 240 python3 -u tools/dbg_race.py $dt 30 $mode > $O/race_${name}_$T.log 2>&1 || { echo "race $name failed"; tail -5 $O/race_${name}_$T.log; return 1; }
  echo "$name: $(grep summary $O/race_${name}_$T.log)"
}
run a16bmixed fp16 other "" DBG_OTHER_DT=mixed && run a32bmixed fp32 other "" DBG_OTHER_DT=mixed
