# round-4 call AB: the packed GN beside bare MFMA loops (f16 / bf16 / f32).
# Usage: bash tools/gpu_r4ab.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for v in pk nopk; do
  for hw in "14 16" "112 128"; do
    for bg in 128 256 512; do
      tag=${v}_bg${bg}_${hw// /x}
      timeout -k 10 150 ./tools/native/gn_repro_$v 300 $bg $hw > $O/gnmf_${T}_$tag.log 2>&1 || { echo "gn_repro $tag failed: $?"; tail -3 $O/gnmf_${T}_$tag.log; exit 1; }
      echo "$tag: $(tail -1 $O/gnmf_${T}_$tag.log)"
    done
  done
done
