# round-4 call AH: long pipelined soaks of the final tree (four model streams,
# 8 hardware queues): every output of every step bit-equal to the serial step.
# Usage: bash tools/gpu_r4ah.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for spec in "fp32 600" "fp16 600" "x6 400"; do
  set -- $spec
  if [ $1 = x6 ]; then DT=fp32; SPLIT=6; else DT=$1; SPLIT=; fi
  DET_SPLIT=$SPLIT GPU_MAX_HW_QUEUES=8 timeout -k 10 500 python3 -u tools/determinism.py $DT $2 32 4 > $O/soak_${1}_$T.log 2>&1 || { echo "soak $1 failed"; tail -3 $O/soak_${1}_$T.log; exit 1; }
  echo "$1: $(tail -1 $O/soak_${1}_$T.log)"
done
