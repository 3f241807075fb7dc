# ROIAlign kernel mode A/B in the bench loop (mdx_policy.roi_mode 4 / 5 / 6),
# interleaved twice, without secondaries.  Usage: bash tools/gpu_ab_roi.sh
O=gpurun_out
mkdir -p $O
B="--no-cpu-baseline --no-secondary --no-roofline"
for r in 1 2; do
  for m in 4 5 6; do
    timeout -k 10 200 python3 -u bench.py $B --roi-mode $m > $O/abroi_${m}_$r.json 2>&1 || exit 1
  done
done
