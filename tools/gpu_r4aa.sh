# round-4 call AA: the packed GN beside the library's register-staged fp16
# convs (f16 MFMA without LDS-DMA), then the x6 pipelined determinism with the
# single-stage kernel.  Usage: bash tools/gpu_r4aa.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out; mkdir -p $O
for v in pk nopk; do
  for hw in "14 16" "112 128"; do
    tag=${v}_${hw// /x}
    BG_CONV_REG=1 timeout -k 10 150 ./tools/native/gn_repro_$v 300 4 $hw > $O/gnreg_${T}_$tag.log 2>&1 || { echo "gn_repro $tag failed: $?"; tail -3 $O/gnreg_${T}_$tag.log; exit 1; }
    echo "$tag: $(tail -1 $O/gnreg_${T}_$tag.log)"
  done
done
DET_SPLIT=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u tools/determinism.py fp32 150 32 3 > $O/det_x6sb_$T.log 2>&1 || { echo "det failed"; tail -3 $O/det_x6sb_$T.log; exit 1; }
tail -1 $O/det_x6sb_$T.log
