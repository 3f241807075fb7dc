# round-4 call J: which co-running work makes the packed-FP32 GN differ in
# the model: the forward on stream A beside (conv) the library's fp16 3x3
# conv, (gn) its GroupNorm, (torch) a torch copy / scale, on stream B.
# Usage: bash tools/gpu_r4j.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for mode in conv gn torch; do
  MDX_LIB_VARIANT=pk MDX_DEBUG_SHADOW=1 timeout -k 10 240 python3 -u tools/dbg_race.py fp16 30 $mode > $O/race_${mode}_$T.log 2>&1 || { echo "race $mode failed"; tail -5 $O/race_${mode}_$T.log; exit 1; }
  echo "$mode: $(grep summary $O/race_${mode}_$T.log)"
done
