# round-4 call R: the packed GN beside the same GN kernels on a small map
# (two forwards' level-5 GN in the same phase), then call P.
# Usage: bash tools/gpu_r4r.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for v in pk nopk; do
  for hw in "14 16 4" "28 32 4"; do
    tag=${v}_${hw// /x}
    GN_BG="$hw" GN_BG_LAUNCHES=40 timeout -k 10 150 ./tools/native/gn_repro_$v 300 32 14 16 > $O/gnsm_${T}_$tag.log 2>&1 || { echo "gn_repro $tag failed: $?"; tail -3 $O/gnsm_${T}_$tag.log; exit 1; }
    echo "$tag: $(tail -1 $O/gnsm_${T}_$tag.log)"
  done
done
bash tools/gpu_r4p.sh $T
