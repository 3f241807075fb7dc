# A/B of bench variants in one box session: bash tools/gpu_ab.sh TAG "args A" "args B" ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
T=$1; shift
i=0
for a in "$@"; do
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 4 --no-cpu-baseline --no-roofline $a > $O/ab${T}_${i}_$rep.json 2>/dev/null || exit 1
  done
  i=$((i+1))
done
