# round-4 call G.  Usage: bash tools/gpu_r4g.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
# GN statistics beside packed-FP32 VALU work and beside the GN kernels
# themselves on another stream, packed and unpacked GN builds
for v in pk nopk; do
  for hw in "14 16" "112 128"; do
    for bg in 16 32 52; do
      tag=${v}_bg${bg}_${hw// /x}
      timeout -k 10 150 ./tools/native/gn_repro_$v 300 $bg $hw > $O/gn_${T}_$tag.log 2>&1 || { echo "gn_repro $tag failed: $?"; tail -3 $O/gn_${T}_$tag.log; exit 1; }
      echo "$tag: $(tail -1 $O/gn_${T}_$tag.log)"; grep -m2 "^rep" $O/gn_${T}_$tag.log
    done
  done
done
