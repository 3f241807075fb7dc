# round-4 call AC: which packed-FP32 instruction forms fault beside 16-bit
# MFMA loops (tools/native/pk_hazard.hip).  Usage: bash tools/gpu_r4ac.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for bg in 0 1 2 3; do
  timeout -k 10 200 ./tools/native/pk_hazard 200 $bg > $O/pkh_${T}_$bg.log 2>&1 || { echo "pk_hazard bg$bg failed: $?"; tail -3 $O/pkh_${T}_$bg.log; exit 1; }
  echo "bg$bg: $(tail -1 $O/pkh_${T}_$bg.log)"
done
