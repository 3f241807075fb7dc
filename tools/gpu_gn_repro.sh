# GroupNorm statistics under concurrency, packed-FP32 build vs not
# (tools/native/gn_repro.hip).  Usage: bash tools/gpu_gn_repro.sh TAG [REPS]
set -o pipefail
T=${1:-x}; R=${2:-400}
O=gpurun_out; mkdir -p $O
for v in nopk pk; do
  for bg in 0 3 1 2; do
    timeout -k 10 120 ./tools/native/gn_repro_$v $R $bg > $O/gn_${T}_${v}_bg$bg.log 2>&1 || { echo "gn_repro_$v bg$bg failed: $?"; exit 1; }
    echo "$v bg$bg: $(tail -1 $O/gn_${T}_${v}_bg$bg.log)"
  done
done
