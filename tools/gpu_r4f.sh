# round-4 call F.  Usage: bash tools/gpu_r4f.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
# GN statistics beside the library's own convs on another stream: fp16 3x3
# (LDS-DMA k_convg) and fp32 3x3 (k_conv_sb), packed and unpacked GN builds
for v in pk nopk; do
  for hw in "14 16" "112 128"; do
    for bg in 4 8; do
      tag=${v}_bg${bg}_${hw// /x}
      timeout -k 10 150 ./tools/native/gn_repro_$v 200 $bg $hw > $O/gn_${T}_$tag.log 2>&1 || { echo "gn_repro $tag failed: $?"; tail -3 $O/gn_${T}_$tag.log; exit 1; }
      echo "$tag: $(tail -1 $O/gn_${T}_$tag.log)"; grep -m2 "^rep" $O/gn_${T}_$tag.log
    done
  done
done
# split-plane serial steps: where the time goes with and without the plane Winograd GEMMs
for m in 0 1; do
  if [ $m = 1 ]; then export MDX_WINO_X6=1; else unset MDX_WINO_X6; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/px6_${T}_$m -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 3 --no-overlap --no-roofline --no-cpu-baseline --no-secondary --no-extract-loop --set mdx_conv_set_fp32_split=6 > $O/px6_${T}_$m.log 2>&1 || { echo "prof x6 $m failed"; tail -3 $O/px6_${T}_$m.log; exit 1; }
  echo "x6 planes=$m"; tail -1 $O/px6_${T}_$m.log | cut -c1-300
done
unset MDX_WINO_X6
